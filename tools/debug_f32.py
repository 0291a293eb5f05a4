"""Debug: small fp32 factorisations through the persistent engine vs the oracle, tile by tile."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpu-tiled-qr-decomposition_amd"))
from conftest import Oracle
import tqr
orc = Oracle()
for (m, n, b) in [(16, 32, 16), (32, 16, 16), (32, 32, 16), (64, 64, 32), (128, 128, 64), (256, 256, 128), (512, 512, 256)]:
    A = orc.randzo(m, n, np.float32, seed=5)
    F_ref, T_ref = orc.factor(A, b)
    F = A.copy()
    T = tqr.geqrt_host(F, b)
    d = np.abs(F.astype(np.float64) - F_ref)
    p, q = m // b, n // b
    bad = [(i, j, float(d[j * b:(j + 1) * b, i * b:(i + 1) * b].max())) for i in range(p) for j in range(q)]
    print(m, n, b, "max", float(d.max()), "tiles:", " ".join(f"({i},{j}):{e:.1e}" for i, j, e in bad[:16]), flush=True)
