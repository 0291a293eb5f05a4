"""Per-tile parity of the HIP tile kernels (through the C ABI) against the reference's outputs
(golden fixtures from oracle/_ref) and, for tile sizes without fixtures, against the oracle.

Tolerances (fp64 arithmetic everywhere on the GPU; the reference rounds in its own order):
  fp64 tiles: max|GPU - ref| <= 1e-12 * max(1, max|ref|)
  fp32 tiles: max|GPU - ref| <= 1e-4  * max(1, max|ref|)   (the reference EPSILON is 1e-3)
"""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden, ptr

pytestmark = pytest.mark.gpu


def tol(dt):
    return 1e-12 if dt == np.float64 else 1e-4


def close(a, b):
    s = max(1.0, float(np.abs(b).max()))
    return float(np.abs(a.astype(np.float64) - b.astype(np.float64)).max()) <= tol(b.dtype) * s


def run_tile(tqr, op, X, b, tau_in=None):
    X = X.copy()
    tau = np.zeros(b, X.dtype) if tau_in is None else tau_in.copy()
    getattr(tqr, f"tile_{op}")(X, b, tau)
    return X, tau


TILES = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "tile_*.npz")))


@pytest.mark.parametrize("name", TILES)
def test_tile_vs_reference(tqr, name):
    g = golden(name)
    X_in, X_out, tau, b = g["X_in"], g["X_out"], g["tau"], int(g["b"])
    op = name.split("_")[1]
    if op in ("geqrt", "tsqrt"):
        X, t = run_tile(tqr, op, X_in, b)
        assert close(t, tau)
    else:
        X, _ = run_tile(tqr, op, X_in, b, tau)
    assert close(X, X_out)


def oracle_tile(oracle, op, X_in, b, tau=None):
    import ctypes
    X = X_in.copy()
    m = X.shape[1]
    es, base, P = X.itemsize, X.ctypes.data, ctypes.c_void_p
    sfx = oracle.sfx(X.dtype)
    w = np.zeros(2 * b, X.dtype)
    t = np.zeros(b, X.dtype) if tau is None else tau
    L = oracle.L
    if op == "geqrt":
        getattr(L, f"oracle_geqrt_{sfx}")(ptr(X), ptr(t), b, b, m, ptr(w))
    elif op == "unmqr":
        getattr(L, f"oracle_unmqr_{sfx}")(P(base + b * m * es), ptr(X), ptr(t), b, b, m)
    elif op == "tsqrt":
        getattr(L, f"oracle_tsqrt_{sfx}")(ptr(X), P(base + b * es), ptr(t), b, b, b, m, ptr(w))
    elif op == "tsmqr":
        getattr(L, f"oracle_tsmqr_{sfx}")(P(base + b * es), P(base + b * m * es), P(base + (b * m + b) * es),
                                          ptr(t), b, b, m)
    return X, t


@pytest.mark.parametrize("b", [16, 32, 64, 128, 256])
@pytest.mark.parametrize("dt", [np.float64, np.float32])
def test_tile_chain_vs_oracle(tqr, oracle, b, dt):
    """GEQRT -> UNMQR, TSQRT -> TSMQR on a 2b x 2b RANDZO block, each step from the oracle's
    previous output, compared with the oracle."""
    X0 = oracle.randzo(2 * b, 2 * b, dt, seed=3 + b)
    Xo, to = oracle_tile(oracle, "geqrt", X0, b)
    Xg, tg = run_tile(tqr, "geqrt", X0, b)
    assert close(tg, to) and close(Xg, Xo)
    Xo2, _ = oracle_tile(oracle, "unmqr", Xo, b, to)
    Xg2, _ = run_tile(tqr, "unmqr", Xo, b, to)
    assert close(Xg2, Xo2)
    Xo3, to3 = oracle_tile(oracle, "tsqrt", Xo2, b)
    Xg3, tg3 = run_tile(tqr, "tsqrt", Xo2, b)
    assert close(tg3, to3) and close(Xg3, Xo3)
    Xo4, _ = oracle_tile(oracle, "tsmqr", Xo3, b, to3)
    Xg4, _ = run_tile(tqr, "tsmqr", Xo3, b, to3)
    assert close(Xg4, Xo4)


@pytest.mark.parametrize("b", [32, 256])
def test_tile_zero_and_unit_columns(tqr, oracle, b):
    """Zero columns (tau = 2, no scaling, qrdecomp.c:1219,1265) and an identity block."""
    X0 = oracle.randzo(2 * b, 2 * b, np.float64, seed=9)
    X0[3, :] = 0.0          # matrix column 3 is zero in every tile row
    X0[b + 5, b:] = 0.0     # column 5 of the lower-left tile zero
    X0[:b, :b] = 0.0
    X0[:b, :b][np.arange(b), np.arange(b)] = 1.0  # tile (0,0) = I
    for op in ("geqrt", "tsqrt"):
        Xo, to = oracle_tile(oracle, op, X0, b)
        Xg, tg = run_tile(tqr, op, X0, b)
        assert close(tg, to) and close(Xg, Xo), op


def test_docudadapp_matches_oracle(tqr, oracle):
    """doCUDADAPP (reference gpucalc.cu:1776): one TSMQR on a 64 x 64 fp32 matrix with
    V = tile (1,0), A = tile (0,1), B = tile (1,1) and tau = the matrix's first 32 entries."""
    import ctypes
    b, ldm = 32, 64
    M = oracle.randzo(64, 64, np.float32, seed=7)
    M[0, :b] = np.linspace(0.5, 1.5, b, dtype=np.float32)  # plausible taus in column 0
    ref = M.copy()
    tau = ref[0, :b].copy()
    P = ctypes.c_void_p
    es = ref.itemsize
    base = ref.ctypes.data
    oracle.L.oracle_tsmqr_s(P(base + b * es), P(base + b * ldm * es), P(base + (b * ldm + b) * es),
                            tau.ctypes.data_as(P), b, b, ldm)
    G = M.copy()
    tqr.lib().doCUDADAPP(G.ctypes.data_as(P))
    assert float(np.abs(G.astype(np.float64) - ref.astype(np.float64)).max()) <= 1e-4 * max(1.0, float(np.abs(ref).max()))
