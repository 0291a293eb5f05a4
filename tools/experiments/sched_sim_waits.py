import sys, os
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))  # tools/
import sched_sim as S
items = S.export_list(256, 64)
for w in (1, 8):
    wt = {}
    t = S.simulate_dist_dyn(items, 256, 64, w, waits=wt)
    print(f"world {w}: {t/1e3:.1f} ms")
    for c in sorted(wt):
        print(f"   {c:28s} {wt[c] / (w * 256) / 1e3:7.2f} ms/WG")
