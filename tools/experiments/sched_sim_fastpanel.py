"""What-if of tools/sched_sim.py: a faster panel (every panel cost scaled by `a`) under the engine's
in-order per-rank dequeue and under dependency-triggered dispatch (simulate_dist_dyn), 1 and 8
ranks. Usage: python tools/sched_sim_fastpanel.py [M] [N] [a ...]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # tools/
import sched_sim as S
M = int(sys.argv[1]) if len(sys.argv) > 1 else 256
N = int(sys.argv[2]) if len(sys.argv) > 2 else 64
scales = [float(x) for x in sys.argv[3:]] or [1.0, 0.5, 0.3]
items = S.export_list(M, N)
P = S.P
for a in scales:
    pp = dict(P, f=P["f"] * a, bt=P["bt"] * a, t=P["t"] * a, io_in=P["io_in"] * a, io_wb=P["io_wb"] * a,
              io_img=P["io_img"] * a)
    t1 = S.simulate_dist(items, M, N, 1, prm=pp)
    t8 = S.simulate_dist(items, M, N, 8, prm=pp)
    d1 = S.simulate_dist_dyn(items, M, N, 1, prm=pp)
    d8 = S.simulate_dist_dyn(items, M, N, 8, prm=pp)
    print(f"panel x{a:.2f}: in-order t1 {t1 / 1e3:6.1f} t8 {t8 / 1e3:6.1f} S {t1 / t8:4.2f} | dynamic t1 {d1 / 1e3:6.1f} "
          f"t8 {d8 / 1e3:6.1f} S {d1 / d8:4.2f}", flush=True)
