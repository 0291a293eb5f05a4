import faulthandler, sys, os, ctypes
faulthandler.enable()
sys.path.insert(0, 'tests'); sys.path.insert(0, 'gpu-tiled-qr-decomposition_amd')
import numpy as np
import tqr
from conftest import Oracle
o = Oracle()
print("lib", tqr.lib().tqr_version(), flush=True)
for (m, n, b, dt) in [(64, 64, 32, np.float64), (128, 128, 64, np.float64), (64, 48, 16, np.float32), (512, 512, 64, np.float64)]:
    A = o.randzo(m, n, dt, 5)
    h = ctypes.c_void_p()
    st = tqr.lib().tqr_plan_create(ctypes.byref(h), m, n, b, 1 if dt == np.float64 else 0)
    print("plan", m, n, b, st, flush=True)
    e, nt, eo, g = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    tqr.lib().tqr_plan_info(h, ctypes.byref(e), ctypes.byref(nt), ctypes.byref(eo), ctypes.byref(g))
    print("info", e.value, nt.value, eo.value, g.value, flush=True)
    F = A.copy()
    T = tqr.geqrt_host(F, b)
    Fr, Tr = o.factor(A, b)
    print(m, n, b, "maxdiff", np.abs(F.astype(np.float64) - Fr).max(), flush=True)
