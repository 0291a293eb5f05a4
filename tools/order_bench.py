"""Time the persistent engine with alternative task orders (tools/sched_sim.py list schedules, set
through tqr_plan_set_tasks) against the built-in order. Usage: python tools/order_bench.py [M tiles]"""
import ctypes, os, sys, time
import numpy as np
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "gpu-tiled-qr-decomposition_amd"))
import sched_sim as S
import tqr
L = tqr.lib()
M = int(sys.argv[1]) if len(sys.argv) > 1 else 64
b = 256
m = n = M * b
A0 = torch.empty((n, m), dtype=torch.float64, device="cuda")
tqr.fill_randzo(A0, m, n, 5)
A = A0.clone()
tau = torch.zeros((M, m), dtype=torch.float64, device="cuda")
pl = tqr.TiledQR(m, n, b, torch.float64)


def timeit(label, reps=5):
    ts = []
    for _ in range(reps + 1):
        A.copy_(A0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pl.execute(A, tau)
        pl.status()
        ts.append(time.perf_counter() - t0)
    ts = sorted(ts[1:])
    print(f"{label:40s} median {ts[len(ts) // 2] * 1e3:7.2f} ms  min {ts[0] * 1e3:7.2f}", flush=True)


timeit("built-in order")
orders = {}
for prio in os.environ.get("PRIOS", "panel").split(","):
    for c in [float(x) for x in os.environ.get("CS", "16").split(",")]:
        prm = dict(S.P, c=c)
        orders[f"greedy prio={prio} c={c}"] = S.to_items(S.greedy_order(M, M, prm=prm, prio=prio))
for label, items in orders.items():
    a = np.ascontiguousarray(items.astype(np.int32)).ravel()
    st = L.tqr_plan_set_tasks(pl.h, a.ctypes.data_as(ctypes.c_void_p), len(items))
    assert st == 0, st
    timeit(label)
