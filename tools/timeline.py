"""Diagnostic: task timeline of the persistent engine (libtqr_fst.so): per factorisation step k,
when its panel and its chains start and end, and how many workgroups hold a task over time.
Usage: python tools/timeline.py [m] [b]"""
import ctypes, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpu-tiled-qr-decomposition_amd"))
import tqr
tqr.LIB_PATH = tqr.LIB_PATH.replace("libtqr.so", os.environ.get("TQR_FST_LIB", "libtqr_fst.so"))
L = tqr.lib()
m = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
b = int(sys.argv[2]) if len(sys.argv) > 2 else 256
dt = torch.float32 if os.environ.get("TQR_FST_DTYPE") == "f32" else torch.float64
A = torch.empty((m, m), dtype=dt, device="cuda")
tau = torch.zeros((m // b, m), dtype=dt, device="cuda")
p = tqr.TiledQR(m, m, b, dt)
for rep in range(2):
    tqr.fill_randzo(A, m, m, 5)
    p.execute(A, tau)
    torch.cuda.synchronize()
eng, nt, est, grid = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
L.tqr_plan_info(p.h, ctypes.byref(eng), ctypes.byref(nt), ctypes.byref(est), ctypes.byref(grid))
n = nt.value
tl = (ctypes.c_ulonglong * (3 * n))()
items = (ctypes.c_int * (4 * n))()
assert L.tqr_debug_task_timeline(p.h, tl, n, items) == 0
T = np.frombuffer(tl, dtype=np.uint64).reshape(n, 3).astype(np.int64)
I = np.frombuffer(items, dtype=np.int32).reshape(n, 4)
# (the fp64 asm chain adds its start's dependency wait in bits 16.. of the workgroup word)
Wst = (T[:, 2] >> 16) / 100.0  # us
T[:, 2] &= 0xffff
if os.environ.get("TQR_TIMELINE_DUMP"):
    np.savez_compressed(os.environ["TQR_TIMELINE_DUMP"], T=T, I=I)
t0 = T[:, 0].min()
s = (T[:, 0] - t0) / 100.0  # us (100 MHz)
e = (T[:, 1] - t0) / 100.0
typ = I[:, 0] & 0xff
k = np.where(typ == 4, I[:, 3] & 0xffff, I[:, 3])
chain = typ == 4
print(f"{m}^2 b={b}: {n} tasks, launch span {e.max() / 1e3:.1f} ms, {grid.value} workgroups")
print(" step  panel start..end (ms)   chains start..end (ms)   chain tasks")
K = m // b
for kk in list(range(0, K, max(1, K // 16))) + [K - 1]:
    pm = (k == kk) & ~chain
    cm = (k == kk) & chain
    ps = f"{s[pm].min() / 1e3:7.2f}..{e[pm].max() / 1e3:7.2f}" if pm.any() else "   -   "
    cs = f"{s[cm].min() / 1e3:7.2f}..{e[cm].max() / 1e3:7.2f}" if cm.any() else "   -   "
    print(f" {kk:4d}  {ps}        {cs}      {cm.sum():5d}")
if Wst.any():
    print(" chain tasks' start wait (dependency spins + barrier), per step range:")
    for lo in range(0, K, max(1, K // 8)):
        cm = chain & (k >= lo) & (k < lo + max(1, K // 8))
        if cm.any():
            print(f"   steps {lo:3d}..{lo + max(1, K // 8) - 1:3d}: {cm.sum():6d} tasks, mean {Wst[cm].mean():7.1f} us, "
                  f"total {Wst[cm].sum() / grid.value / 1e3:6.2f} ms per workgroup")
# workgroups holding a task, per 5 % of the span
span = e.max()
print(" occupancy (mean workgroups holding a task) per 5 % of the launch:")
edges = np.linspace(0, span, 21)
occ = []
for a0, a1 in zip(edges[:-1], edges[1:]):
    ov = np.clip(np.minimum(e, a1) - np.maximum(s, a0), 0, None).sum() / (a1 - a0)
    occ.append(ov)
print("  " + " ".join(f"{o:5.0f}" for o in occ))
# panel members of a few steps: start/end per member
for kk in (0, 1, 16):
    pm = np.where((k == kk) & ~chain)[0]
    order = pm[np.argsort(I[pm, 1])]
    rows = [f"{I[x, 1]}:{s[x] / 1e3:.2f}-{e[x] / 1e3:.2f}" for x in order[:: max(1, len(order) // 12)]]
    print(f" step {kk} members (tile row: start-end ms): " + " ".join(rows))
# every task of the last N steps in start order (TQR_TIMELINE_TAIL=N): the tail's critical path
NT = int(os.environ.get("TQR_TIMELINE_TAIL", "0"))
if NT:
    print(f" tasks of steps >= {K - NT} (start..end ms, workgroup, task):")
    sel = np.where(k >= K - NT)[0]
    for x in sel[np.argsort(s[sel])]:
        if chain[x]:
            i0, i1 = I[x, 1] & 0xffff, I[x, 1] >> 16
            desc = f"CHAIN k={k[x]} j={I[x, 2]} strip={(I[x, 0] >> 8) & 0xff} seg={I[x, 3] >> 16} rows {i0}..{i1 - 1}"
        else:
            desc = f"PANEL type={typ[x]} k={k[x]} row={I[x, 1]}"
        print(f"  {s[x] / 1e3:8.3f}..{e[x] / 1e3:8.3f}  wg {T[x, 2]:3d}  {desc}")
