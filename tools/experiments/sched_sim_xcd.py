"""What-if of tools/sched_sim.py for ONE GPU: XCD affinity — the tasks of tile column j (its panel,
its chains) dequeued only by the 32 workgroups of XCD x(j) (the multi-GPU partition with 8
"ranks" of 32 workgroups, no forwarding: images are read in place), so that strips and head rows
could be stored write-back into that XCD's L2 instead of write-through (a cheaper element
hand-over: e_ld / e_st scaled by `h`). Usage: python tools/sched_sim_xcd.py [M] [N] [h ...]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # tools/
import sched_sim as S
M = int(sys.argv[1]) if len(sys.argv) > 1 else 64
N = int(sys.argv[2]) if len(sys.argv) > 2 else 64
hs = [float(x) for x in sys.argv[3:]] or [1.0, 0.5, 0.25]
items = S.export_list(M, N)
base = S.simulate_dist(items, M, N, 1)
print(f"{M}x{N} tiles: one queue, 256 workgroups: {base / 1e3:.1f} ms")
for h in hs:
    prm = dict(S.P, W=32, e_ld=S.P["e_ld"] * h, e_st=S.P["e_st"] * h)
    t = S.simulate_dist(items, M, N, 8, prm=prm, fwd_peer=0.0, hop=0.0)
    prm1 = dict(S.P, e_ld=S.P["e_ld"] * h, e_st=S.P["e_st"] * h)
    t1 = S.simulate_dist(items, M, N, 1, prm=prm1)
    print(f"  element hand-over x{h:.2f}: per-XCD queues {t / 1e3:.1f} ms; one queue with that hand-over {t1 / 1e3:.1f} ms", flush=True)
