"""Chain segment length (TQR_SEGLEN) in the multi-GPU model (tools/sched_sim.py simulate_dist):
makespan and S(world) per segment length, with a per-segment cost (TQR_SIM_SEG us, default 20:
calibrated on one MI355X, 65536x16384 at segment length 2 vs 8 = 635.3 vs 607.6 ms, i.e. 27.7 ms
for ~356k extra segments on 256 workgroups). Usage: python tools/sched_sim_seglen.py [M] [N] [seglen ...]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # tools/
import sched_sim as S
M = int(sys.argv[1]) if len(sys.argv) > 1 else 256
N = int(sys.argv[2]) if len(sys.argv) > 2 else 64
sls = [int(x) for x in sys.argv[3:]] or [8, 4, 3, 2]
seg = float(os.environ.get("TQR_SIM_SEG", "20"))
prm = dict(S.P, seg=seg)
print(f"per-segment cost {seg} us")
for sl in sls:
    items = S.export_list(M, N, seglen=sl)
    t1 = S.simulate_dist(items, M, N, 1, prm=prm)
    line = f"seglen {sl}: t1 {t1 / 1e3:6.1f} ms"
    for w in (2, 4, 8):
        tw = S.simulate_dist(items, M, N, w, prm=prm)
        line += f", t{w} {tw / 1e3:6.1f} (S {t1 / tw:4.2f})"
    print(line, flush=True)
