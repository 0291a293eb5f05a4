"""Diagnostic: activity breakdown of the persistent engine k_flow (libtqr_fst.so, per-workgroup
s_memrealtime sums, flow.hpp FST categories). Usage: python tools/flowstamps.py [m] [n] [b]"""
import ctypes, os, sys, time
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpu-tiled-qr-decomposition_amd"))
import tqr
tqr.LIB_PATH = tqr.LIB_PATH.replace("libtqr.so", os.environ.get("TQR_FST_LIB", "libtqr_fst.so"))
L = tqr.lib()
m = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
n = int(sys.argv[2]) if len(sys.argv) > 2 else m
b = int(sys.argv[3]) if len(sys.argv) > 3 else 256
dt = torch.float32 if os.environ.get("TQR_FST_DTYPE") == "f32" else torch.float64
A = torch.empty((n, m), dtype=dt, device="cuda")
tau = torch.zeros((min(m, n) // b, m), dtype=dt, device="cuda")
p = tqr.TiledQR(m, n, b, dt)
for rep in range(2):
    tqr.fill_randzo(A, m, n, 5)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    p.execute(A, tau)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
gridv = ctypes.c_int()
L.tqr_plan_info(p.h, None, None, None, ctypes.byref(gridv))
nb = gridv.value  # workgroups of the launch (ShapeW4: two per CU)
shape = os.environ.get("TQR_FLOW_SHAPE", "w8") if dt == torch.float64 else "w8"
NW = 4 if shape in ("w4", "r") else 8  # waves per workgroup (r: the resident form, b = 256)
IB = 16 if shape == "w4" else 32  # reflectors per group
NC = 24
st = (ctypes.c_ulonglong * (NC * nb))()
assert L.tqr_debug_flow_stamps(st, nb) == 0
names = ["chain Rc wait in-elem other", "panel waits", "chain head-row store", "chain phase 1 Z (+DMA)",
         "chain strip I/O+publish", "panel_factor", "dequeue/dispatch/exit", "chain drain+barrier",
         "chain Tc waits", "chain Ac waits", "panel I/O+images", "panel build_t", "panel trail MFMA+publish", "chain phase 2", "chain next-head load", "chain W + head update", "panel trail loads", "panel trail stores",
         "chain Rc wait @start la-col", "chain Rc wait @start other", "chain Rc wait in-elem la-col", "chain own-memory drain @group>0", "chain own-memory drain @group0", "panel fwd to peers (multi-GPU)"]
tot = [sum(st[w * NC + c] for w in range(nb)) for c in range(NC)]
allt = sum(tot)
print(f"{m}x{n} b={b}: wall {ms:.1f} ms; {nb} workgroups; sum of stamps {allt / nb / 1e5:.1f} ms per WG")
pt, q = m // b, n // b
npanel = sum(pt - k for k in range(min(pt, q)))
ng = b // min(b, IB)
for c, nm in ((5, "panel_factor"), (11, "build_t"), (12, "trailing"), (10, "panel I/O")):
    print(f"  per panel group ({npanel * ng} groups): {nm:14s} {tot[c] / (npanel * ng) / 100:7.2f} us")
for c in range(NC):
    print(f"  {names[c]:24s} {tot[c] / nb / 1e5:8.2f} ms/WG  {100.0 * tot[c] / allt:5.1f}%")
WSL = 8
ws = (ctypes.c_ulonglong * (8 * WSL * nb))()  # (g_wst holds 8 wave slots per workgroup)
if hasattr(L, "tqr_debug_flow_wave_stamps") and L.tqr_debug_flow_wave_stamps(ws, nb) == 0:
    # (the asm chains: "phase1" is the whole group statement, slot 5 the task-start dependency wait
    # (spins + barrier), slot 6 the task end (element end, drain barrier, publishes))
    asm = os.environ.get("TQR_CHAIN_ASM", "2") != "0"
    wn = ["drain", "barrier", "pre-sync", "post-sync", "body" if asm else "phase1", "tstart" if asm else "head I/O",
          "tend" if asm else "phase2", "tail"]
    print("  per-wave sums (ms/WG): " + " | ".join(f"{n:>9s}" for n in wn))
    for w in range(NW):
        v = [sum(ws[b * 8 * WSL + WSL * w + c] for b in range(nb)) / nb / 1e5 for c in range(WSL)]
        print(f"    wave {w}:            " + " | ".join(f"{x:9.2f}" for x in v) + f" | sum {sum(v):7.2f}")
