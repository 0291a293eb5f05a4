"""Diagnostic: phase breakdown of the TSQRT panel kernel (libtqr_stamps.so, s_memtime sums)."""
import ctypes, os, sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpu-tiled-qr-decomposition_amd"))
import tqr
tqr.LIB_PATH = tqr.LIB_PATH.replace("libtqr.so", "libtqr_stamps.so")
L = tqr.lib()
m = n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
b = 256
A = torch.empty((n, m), dtype=torch.float64, device="cuda"); tqr.fill_randzo(A, m, n, 5)
tau = torch.zeros((m // b, m), dtype=torch.float64, device="cuda")
p = tqr.TiledQR(m, n, b, torch.float64)
p.execute(A, tau); torch.cuda.synchronize()
st = (ctypes.c_ulonglong * 16)()
L.tqr_debug_stamps(st, 1)
tqr.fill_randzo(A, m, n, 5); p.execute(A, tau); torch.cuda.synchronize()
L.tqr_debug_stamps(st, 0)
ntsqrt = sum((m // b - k - 1) for k in range(n // b))
names = ["stage", "panel_factor", "writeback", "build_t", "trailing"]
tot = sum(st[i] for i in range(5))
for i, nm in enumerate(names):
    print(f"{nm:14s} {st[i] / ntsqrt / 100:9.1f} us/TSQRT (s_memtime @100MHz)  {100 * st[i] / tot:5.1f}%")
nsteps = ntsqrt * 256  # reflector steps (all panel tasks incl. GEQRT are counted in pstamps)
ngeq = n // b
nsteps_all = (ntsqrt + ngeq) * 256
pn = ["products+reduce", "barrier wait", "exchange+scalars", "update"]
for i, nm in enumerate(pn):
    print(f"panel step {nm:18s} {st[8 + i] / nsteps_all:8.0f} cycles/step")
