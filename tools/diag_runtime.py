"""Diagnostic: which libamdhip64 gets loaded when torch and libtqr share a process."""
import ctypes, os, sys
order = sys.argv[1]
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpu-tiled-qr-decomposition_amd"))
def maps():
    return sorted({l.split()[-1] for l in open("/proc/self/maps") if "amdhip64" in l})
if order == "torch-first":
    import torch
    print("torch cuda", torch.cuda.is_available(), torch.cuda.device_count())
    import tqr
    L = tqr.lib()
else:
    import tqr
    L = tqr.lib()
    import numpy as np
    A = np.random.rand(64, 64)
    print("tqr host call", L.tqr_dgeqrt_host(A.ctypes.data_as(ctypes.c_void_p), None, 64, 64, 64, 32))
    import torch
    print("torch cuda", torch.cuda.is_available(), torch.cuda.device_count())
print(order, maps())
if order == "torch-first":
    import torch
    x = torch.zeros((64, 64), dtype=torch.float64, device="cuda")
    tau = torch.zeros((2, 64), dtype=torch.float64, device="cuda")
    tqr.fill_randzo(x, 64, 64, 5)
    p = tqr.TiledQR(64, 64, 32, torch.float64)
    p.execute(x, tau)
    torch.cuda.synchronize()
    print("ok", float(x.abs().sum()))
