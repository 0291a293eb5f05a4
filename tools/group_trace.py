"""Diagnostic: per-group timeline of workgroup 0's chain tasks (libtqr_fst.so, flow.hpp GTR marks):
for every reflector group and wave, when it reached the sync point, left it, and ran phase 1, the
head I/O and phase 2 — who arrives last at the group barrier, how long the pair of waves on each
SIMD keeps the MFMA pipe fed, where the group time goes. Usage: python tools/group_trace.py [m] [b]"""
import ctypes, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpu-tiled-qr-decomposition_amd"))
import tqr
tqr.LIB_PATH = tqr.LIB_PATH.replace("libtqr.so", os.environ.get("TQR_FST_LIB", "libtqr_fst.so"))
L = tqr.lib()
m = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
b = int(sys.argv[2]) if len(sys.argv) > 2 else 256
dt = torch.float32 if os.environ.get("TQR_FST_DTYPE") == "f32" else torch.float64
A = torch.empty((m, m), dtype=dt, device="cuda")
tau = torch.zeros((m // b, m), dtype=dt, device="cuda")
p = tqr.TiledQR(m, m, b, dt)
for rep in range(2):
    tqr.fill_randzo(A, m, m, 5)
    p.execute(A, tau)
    torch.cuda.synchronize()
NGR = 4096
buf = (ctypes.c_ulonglong * (2 * NGR * 64))()
assert L.tqr_debug_group_trace(buf, NGR) == 0
T = np.frombuffer(buf, dtype=np.uint64)[:NGR * 64].reshape(NGR, 8, 8).astype(np.int64)
XT = np.frombuffer(buf, dtype=np.uint64)[NGR * 64:].reshape(NGR, 8, 8).astype(np.int64)
tag = T[:, 0, 7]
valid = (T[:, :, 2] > 0).all(axis=1)
n = int(valid.sum())
T = T[:n].astype(np.float64)
XT = XT[:n].astype(np.float64)
tag = tag[:n]
g_in = tag & 0xff
us = lambda x: x / 100.0  # s_memrealtime: 100 MHz
arr = T[:, :, 1]      # before the sync point (after polls)
ext = T[:, :, 2]      # after it
p1 = T[:, :, 4] - T[:, :, 3]
hd = T[:, :, 5] - T[:, :, 4]
p2 = T[:, :, 6] - T[:, :, 5]
post = T[:, :, 3] - T[:, :, 2]
last = arr.argmax(axis=1)
gap = ext.min(axis=1) - arr.max(axis=1)
dur = np.diff(ext.min(axis=1))
print(f"{n} groups traced (workgroup 0); median group {us(np.median(dur)):.2f} us (mean {us(dur.mean()):.2f})")
print("last wave to reach the sync point (count per wave):", np.bincount(last, minlength=8).tolist())
print(f"last arrival -> exit (drain + barrier): median {us(np.median(gap)):.2f} us, mean {us(gap.mean()):.2f}")
for w in range(8):
    print(f"  wave {w}: phase1 {us(np.median(p1[:, w])):6.2f}  head/W {us(np.median(hd[:, w])):5.2f}  phase2 {us(np.median(p2[:, w])):6.2f}"
          f"  post-sync {us(np.median(post[:, w])):5.2f}  wait at sync (arrival -> exit) {us(np.median(ext[:, w] - arr[:, w])):5.2f} us (median)")
# per SIMD (waves s, s+4): span from the exit to the later wave's phase-2 end, and each wave's MFMA share
for s in range(4):
    span = np.maximum(T[:, s, 6], T[:, s + 4, 6]) - ext.min(axis=1)
    print(f"  SIMD {s}: exit -> both waves' phase 2 done: median {us(np.median(span)):.2f} us")
for gi in range(8):
    sel = g_in[:-1] == gi
    if sel.any():
        print(f"  group {gi} of an element: median duration {us(np.median(dur[sel])):.2f} us, last arrival wave {np.bincount(last[:-1][sel], minlength=8).argmax()}")
# hand-over groups: phase-2 progress at pairs 0, 8, 16, 24 and the end (relative to the group's sync exit)
h7 = np.where((XT[:, :, 0] > 0).all(axis=1))[0]
if len(h7):
    e0 = ext[h7].min(axis=1)
    print(f"hand-over phase 2 ({len(h7)} groups), marks at pairs 0/8/16/24/end, us after the sync exit (median):")
    for w in range(8):
        print(f"  wave {w}: " + " ".join(f"{us(np.median(XT[h7, w, q] - e0)):6.2f}" for q in range(5)) +
              f"   | phase 2 end {us(np.median(T[h7, w, 6] - e0)):6.2f}")
if os.environ.get("TQR_GTR_DUMP"):
    np.savez_compressed(os.environ["TQR_GTR_DUMP"], T=T, tag=tag, XT=XT)
