"""Diagnostic: column-norm check of the fp64 engine per tile column at several sizes (b = 256),
and at the smallest an elementwise comparison with the oracle (first wrong tiles). Usage:
python tools/debug_shape.py [sizes...]  (TQR_FLOW_SHAPE selects the engine shape)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gpu-tiled-qr-decomposition_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import tqr  # noqa: E402

b = int(os.environ.get("TQR_DBG_B", "256"))
sizes = [int(x) for x in sys.argv[1:]] or [2048, 4096, 8192, 16384]
for n in sizes:
    m = n
    A0 = torch.empty((n, m), dtype=torch.float64, device="cuda")
    tqr.fill_randzo(A0, m, n, 5)
    plan = tqr.TiledQR(m, n, b, torch.float64)
    want_oracle = n <= int(os.environ.get("TQR_DBG_ORACLE_MAX", "4096"))
    F_ref = T_ref = None
    for rep in range(int(os.environ.get("TQR_DBG_RUNS", "3"))):
        A = A0.clone()
        tau = torch.zeros((n // b, m), dtype=torch.float64, device="cuda")
        plan.execute(A, tau)
        plan.status()
        R = torch.triu(A.T).T
        rel = ((torch.linalg.vector_norm(A0, dim=1) - torch.linalg.vector_norm(R, dim=1)).abs()
               / torch.linalg.vector_norm(A0, dim=1))
        badcols = sorted(set((torch.nonzero(rel > 1e-10).flatten() // b).tolist()))
        print(f"{n}^2 run {rep}: max col-norm err {rel.max().item():.3e}, bad tile columns {badcols[:20]}"
              f"{' ...' if len(badcols) > 20 else ''} ({len(badcols)})", flush=True)
        if want_oracle and (badcols or rep == 0):
            if F_ref is None:
                from conftest import Oracle
                F_ref, T_ref = Oracle().factor(A0.cpu().numpy(), b, threads=16)
            F = A.cpu().numpy()
            D = np.abs(F - F_ref).reshape(n // b, b, m // b, b).max(axis=(1, 3))  # [tile col j][tile row i]
            bad = np.argwhere(D > 1e-9)
            # earliest in DAG order: the tile (i, j) finished at step min(i, j) — the smallest step first
            order = sorted(((min(int(i), int(j)), int(i), int(j)) for j, i in bad))
            print(f"  vs oracle: max {D.max():.3e}; wrong tiles (step, i, j) earliest first: {order[:16]} ({len(bad)})",
                  flush=True)
            tc = tau.cpu().numpy()
            dt_ = np.array([np.abs(tc[k, k * b:] - T_ref[k * b, k * b:]).max() for k in range(n // b)])
            wp = np.nonzero(dt_ > 1e-9)[0]
            print(f"  tau: wrong panels {wp[:12].tolist()}", flush=True)
    del A0, A, plan
    torch.cuda.empty_cache()
