"""Diagnostic: device time per factorisation of the persistent engine (no correctness check — for
A/B timing of engine variants while one of them is being debugged). Usage:
python tools/time_engine.py [n] [reps] [f32]   (TQR_FLOW_SHAPE / TQR_* knobs from the environment)"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gpu-tiled-qr-decomposition_amd"))
import tqr  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
dt = torch.float32 if len(sys.argv) > 3 and sys.argv[3] == "f32" else torch.float64
b = 256
A0 = torch.empty((n, n), dtype=dt, device="cuda")
tqr.fill_randzo(A0, n, n, 5)
As = [A0.clone() for _ in range(reps + 1)]
tau = torch.zeros((n // b, n), dtype=dt, device="cuda")
plan = tqr.TiledQR(n, n, b, dt)
plan.execute(As[0], tau)
plan.status()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s = torch.cuda.current_stream()
e0.record(s)
for r in range(reps):
    plan.execute(As[r + 1], tau, stream=s.cuda_stream)
e1.record(s)
torch.cuda.synchronize()
plan.status()
ms = e0.elapsed_time(e1) / reps
print(f"{os.environ.get('TQR_FLOW_SHAPE', 'default')} {n}^2 {str(dt)[6:]}: {ms:.2f} ms per factorisation, "
      f"{tqr.flops(n, n) / ms / 1e9:.1f} TF/s", flush=True)
