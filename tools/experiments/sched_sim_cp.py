import sys
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))  # tools/
import sched_sim as S
items = S.export_list(256, 64)
P = S.P
a = 0.3
fast = dict(P, f=P["f"] * a, bt=P["bt"] * a, t=P["t"] * a, io_in=P["io_in"] * a, io_wb=P["io_wb"] * a, io_img=P["io_img"] * a)
for name, prm, fine in (("base", P, None), ("fine", P, (2.0, 2.0)), ("panel x0.3", fast, None), ("fine+panel x0.3", fast, (1.0, 1.0))):
    inf = dict(prm, W=20000)
    cp8 = S.simulate_dist(items, 256, 64, 8, prm=inf, fine=fine)
    cp1 = S.simulate_dist(items, 256, 64, 1, prm=inf, fine=fine)
    print(f"{name:18s}: critical path (unbounded workgroups) 1 rank {cp1/1e3:6.1f} ms, 8 ranks {cp8/1e3:6.1f} ms", flush=True)
