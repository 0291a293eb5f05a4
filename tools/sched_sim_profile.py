"""Utilisation profile of the multi-GPU model (tools/sched_sim.py simulate_dist): per 5 ms bin, the
mean number of busy workgroups per rank (of 256) and the step range of the tasks running.
Usage: python tools/sched_sim_profile.py [M] [N] [world]"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import sched_sim as S
M = int(sys.argv[1]) if len(sys.argv) > 1 else 256
N = int(sys.argv[2]) if len(sys.argv) > 2 else 64
w = int(sys.argv[3]) if len(sys.argv) > 3 else 8
items = S.export_list(M, N)
tr = []
span = S.simulate_dist(items, M, N, w, trace=tr)
tr = np.array(tr, dtype=np.float64)  # rank, t0, end, typ, k
bins = np.arange(0, span + 5000, 5000)
print(f"{w} ranks, makespan {span / 1e3:.1f} ms; busy workgroups per rank (mean over the bin) and steps running")
for b0, b1 in zip(bins[:-1], bins[1:]):
    busy = np.zeros(w)
    for r in range(w):
        sel = tr[:, 0] == r
        ov = np.clip(np.minimum(tr[sel, 2], b1) - np.maximum(tr[sel, 1], b0), 0, None)
        busy[r] = ov.sum() / (b1 - b0)
    run = tr[(tr[:, 1] < b1) & (tr[:, 2] > b0)]
    ks = (int(run[:, 4].min()), int(run[:, 4].max())) if len(run) else (-1, -1)
    print(f"  {b0 / 1e3:6.1f}-{b1 / 1e3:6.1f} ms: " + " ".join(f"{x:5.0f}" for x in busy) + f"   steps {ks[0]}-{ks[1]}")
