"""Per-tile-op microbenchmark (the reference's testDAPP, gpucalc.cu:1706-1774,
generalised): batched independent TSMQR (DAPP) / UNMQR (SAPP) tile updates through the C ABI
tqr_tile_batch, one launch of the update kernel per (dtype, type, b), swept over the tile size.
Reports device time (HIP events) and GFLOP/s (TSMQR 4b^3, UNMQR 2b^3 flop per tile), and checks
copy 0 of each batch against copy nblocks-1 (all copies get the same update).
Usage: python tools/tile_bench.py [min_tiles]   (JSON lines on stdout)"""
import ctypes, json, os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpu-tiled-qr-decomposition_amd"))
import tqr

L = tqr.lib()
vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)
min_tiles = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
rng = np.random.default_rng(5)
for dt, code, name in ((np.float64, 1, "f64"), (np.float32, 0, "f32")):
    for b in (16, 32, 64, 128, 256):
        for typ, tname, rows, fl in ((3, "TSMQR", 2, 4.0), (1, "UNMQR", 1, 2.0)):  # DAPP, SAPP (gridscheduler.h)
            nb = max(min_tiles, 1)
            # keep the batch's device footprint moderate (out is host-side: nb blocks)
            nb = min(nb, max(64, (1 << 30) // (rows * b * b * np.dtype(dt).itemsize)))
            blk = rng.uniform(-1, 1, (b, rows * b)).astype(dt)      # column-major [A; B] (ld rows*b)
            # column-major b x b V as a (b, b) C array V[col, row]; SAPP: unit-lower V (zeros on and
            # above the diagonal in storage, the unit diagonal implicit)
            V = np.triu(rng.uniform(-1, 1, (b, b)), 1).astype(dt) if typ == 1 else rng.uniform(-0.5, 0.5, (b, b)).astype(dt)
            V /= np.sqrt(b)
            # orthogonal reflectors (tau = 2 / (1 + |v|^2), v = [e_j; V column]): norm-preserving
            # updates, so the fp32 batch stays finite at b = 256 (random taus overflowed it)
            Vd = V.astype(np.float64)
            tau = (2.0 / (1.0 + (Vd * Vd).sum(axis=0 if typ == 1 else 0))).astype(dt)
            out = np.zeros((nb * b, rows * b), dt)
            ms = ctypes.c_float()
            best = None
            rc = 0
            for rep in range(3):
                rc = L.tqr_tile_batch(code, typ, b, nb, vp(V), b, vp(tau), vp(blk), rows * b, vp(out), rows * b,
                                      ctypes.byref(ms))
                # a batch beyond the 32-bit offsets of tqr_tile_batch's device matrix is rejected
                # (TQR_EINVAL, before any launch): halve it until it fits
                while rc == -1 and rep == 0 and nb > 64:
                    nb //= 2
                    out = out[:nb * b]
                    rc = L.tqr_tile_batch(code, typ, b, nb, vp(V), b, vp(tau), vp(blk), rows * b, vp(out), rows * b,
                                          ctypes.byref(ms))
                if rc != 0:
                    break
                best = ms.value if best is None else min(best, ms.value)
            if rc != 0:
                print(json.dumps({"dtype": name, "op": tname, "b": b, "tiles": nb, "status": rc}), flush=True)
                continue
            same = float(np.abs(out[:b] - out[(nb - 1) * b:]).max())
            gf = fl * b ** 3 * nb / (best * 1e-3) / 1e9
            print(json.dumps({"dtype": name, "op": tname, "b": b, "tiles": nb, "ms": round(best, 4),
                              "gflops": round(gf, 1), "copies_identical": same == 0.0, "finite": bool(np.isfinite(out).all())}), flush=True)
