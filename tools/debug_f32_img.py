"""Debug: the fp32 chain's operand images (VA, VB, TP) of one GEQRT group vs numpy."""
import ctypes, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpu-tiled-qr-decomposition_amd"))
from conftest import Oracle
import tqr
orc = Oracle()
L = tqr.lib()
m, n, b = 16, 32, 16
A = orc.randzo(m, n, np.float32, seed=5)
F_ref, T_ref = orc.factor(A, b)
dA = torch.from_numpy(A).cuda()
tau = torch.zeros((1, m), dtype=torch.float32, device="cuda")
pl = tqr.TiledQR(m, n, b, torch.float32)
pl.execute(dA, tau)
pl.status()
F = dA.cpu().numpy()
print("tile(0,1) err", np.abs(F[16:32] - F_ref[16:32]).max(), " tile(0,0) err", np.abs(F[:16] - F_ref[:16]).max())
buf = np.zeros(1 << 16, dtype=np.uint8)
nb = L.tqr_plan_debug_workspace(pl.h, 0, buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes)
W = buf[:nb].view(np.float32)
print("workspace bytes", nb)
VAimg, VBimg, TPimg = W[:256], W[256:512], W[512:768]
# expected: explicit unit-lower V of tile (0,0) from the GPU result, T from V and tau
Fm = F.T  # (m, n) matrix
V = np.tril(Fm[:16, :16].astype(np.float64), -1) + np.eye(16)
t = tau.cpu().numpy()[0, :16].astype(np.float64)
G = V.T @ V
U = np.diag(1 / t) + np.triu(G, 1)
T = np.linalg.inv(U)
sig = lambda y: 4 * (y & 3) + (y >> 2)
eVA = np.zeros(256); eVB = np.zeros(256); eTP = np.zeros(256)
for l in range(64):
    x, y = l >> 4, l & 15
    for r in range(4):
        eVA[l * 4 + r] = V[4 * x + r, sig(y)]
        eVB[l * 4 + r] = V[sig(y), 4 * x + r]
        eTP[l * 4 + r] = -T[4 * x + r, sig(y)]
print("VA err", np.abs(VAimg - eVA).max(), "VB err", np.abs(VBimg - eVB).max(), "TP err", np.abs(TPimg - eTP).max())
print("VA[:8]", VAimg[:8], "exp", eVA[:8])
print("TP[:8]", TPimg[:8], "exp", eTP[:8])
# emulate the update with the images (numpy) and compare with the GPU tile (0,1)
C0 = A.T[:16, 16:32].astype(np.float64)
Cexp = C0 + V @ (-T.T @ (V.T @ C0))
print("numpy Q^T C vs oracle", np.abs(Cexp - F_ref.T[:16, 16:32]).max(), " GPU vs numpy", np.abs(F.T[:16, 16:32] - Cexp).max())
