"""Round-6 diagnostic: where a candidate library's factorisation differs from the oracle.

  TQR_LIB=libX.so python tools/experiments/rt_diag.py [reps]
Prints, per shape and repetition, the max error and the (tile row, tile column, 32-column group)
cells whose error exceeds the fp64 tolerance (tests/test_gpu_factor.py). Test infrastructure: it
runs the oracle as the checker only."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "gpu-tiled-qr-decomposition_amd"))
from conftest import Oracle  # noqa: E402
import tqr  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
orc = Oracle()
for m, n in ((2048, 512), (4096, 512), (2048, 1024)):
    b = 256
    A = orc.randzo(m, n, np.float64, seed=5)
    F_ref, T_ref = orc.factor(A, b, threads=8)
    tol = 1e-11 * max(1.0, float(np.abs(F_ref).max()))
    for r in range(reps):
        F = A.copy()
        T = tqr.geqrt_host(F, b)
        E = np.abs(F - F_ref)  # (n, m): row = matrix column
        bad = []
        for j in range(n // b):
            for g in range(b // 32):
                for i in range(m // b):
                    e = float(E[j * b + 32 * g:j * b + 32 * g + 32, i * b:(i + 1) * b].max())
                    if e > tol:
                        bad.append((i, j, g, f"{e:.1e}"))
        print(f"{m}x{n} rep {r}: max {float(E.max()):.2e} tau {float(np.abs(T - T_ref).max()):.1e} "
              f"bad cells {len(bad)} first {bad[:12]}", flush=True)
