"""What-if of tools/sched_sim.py: chain segments spread over the ranks ((j + segment) % world)
instead of following their tile column's owner, every cross-rank strip / head-row hand-over
charged a flag hop plus a 256 KiB xGMI copy. Usage: python tools/sched_sim_2d.py [M] [N]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # tools/
import sched_sim as S
M = int(sys.argv[1]) if len(sys.argv) > 1 else 256
N = int(sys.argv[2]) if len(sys.argv) > 2 else 64
items = S.export_list(M, N)
t1 = S.simulate_dist(items, M, N, 1)
for w in (2, 4, 8):
    tc = S.simulate_dist(items, M, N, w)
    t2 = S.simulate_dist(items, M, N, w, part="2d")
    print(f"{w} ranks: column partition {tc / 1e3:6.1f} ms (S {t1 / tc:4.2f}); segments spread {t2 / 1e3:6.1f} ms (S {t1 / t2:4.2f})", flush=True)
