import sys, os, numpy as np
sys.path.insert(0, 'tests'); sys.path.insert(0, 'gpu-tiled-qr-decomposition_amd')
from conftest import Oracle
import tqr
o = Oracle()
m = n = 512; b = 128
for kind in ["row77", "col300", "both"]:
    A = o.randzo(m, n, np.float64, seed=2)
    if kind in ("row77", "both"): A[:, 77] = 0.0
    if kind in ("col300", "both"): A[300, :] = 0.0
    F_ref, T_ref = o.factor(A, b)
    F = A.copy(); T = tqr.geqrt_host(F, b)
    d = np.abs(F - F_ref)
    j, i = np.unravel_index(np.argmax(d), d.shape)
    bad = np.argwhere(d > 1e-9)
    first = bad[np.lexsort((bad[:, 1], bad[:, 0]))][:5] if len(bad) else []
    print(kind, "maxdiff", d.max(), "at row", i, "col", j, "nbad", len(bad), "first bad (col,row)", [tuple(x) for x in first])
    td = np.abs(T - T_ref); print("  tau maxdiff", td.max(), np.argwhere(td > 1e-9)[:5].tolist())
# tile-level: zero row inside a GEQRT tile
for bb in (32, 128):
    X0 = o.randzo(2*bb, 2*bb, np.float64, seed=9)
    X0[:, 7] = 0.0
    X = X0.copy(); t = np.zeros(bb); tqr.tile_geqrt(X, bb, t)
    import ctypes
    Xo = X0.copy(); to = np.zeros(bb); w = np.zeros(2*bb)
    P = ctypes.c_void_p
    o.L.oracle_geqrt_d(Xo.ctypes.data_as(P), to.ctypes.data_as(P), bb, bb, 2*bb, w.ctypes.data_as(P))
    print("tile geqrt zero-row b", bb, np.abs(X - Xo).max(), np.abs(t - to).max())
