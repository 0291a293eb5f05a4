"""The oracle (CPU restatement) pinned against the reference's own outputs.

tests/golden/* were produced by tests/golden/make_golden.py from oracle/_ref (the reference
host code compiled from /root/reference). Every comparison here is bit-exact.
"""
import glob
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden, ptr, ref_lib


def test_manifest():
    lines = open(os.path.join(GOLDEN, "MANIFEST.md5")).read().split("\n")
    for ln in filter(None, lines):
        h, nm = ln.split()
        assert hashlib.md5(open(os.path.join(GOLDEN, nm), "rb").read()).hexdigest() == h, nm


FACTOR = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "factor_*.npz")))


@pytest.mark.parametrize("name", FACTOR)
def test_oracle_factor_bitexact(oracle, name):
    g = golden(name)
    A, F, T, b = g["A"], g["F"], g["T"], int(g["b"])
    n, m = A.shape
    if name.endswith("_randzo.npz"):  # the input generator is pinned too
        assert np.array_equal(oracle.randzo(m, n, A.dtype, int(g["seed"])), A)
    F1, T1 = oracle.factor(A, b)
    assert np.array_equal(F1.view(np.uint8), F.view(np.uint8))
    assert np.array_equal(T1.view(np.uint8), T.view(np.uint8))
    F2, T2 = oracle.factor(A, b, threads=4)  # any topological order: same bits
    assert np.array_equal(F2, F) and np.array_equal(T2, T)


@pytest.mark.parametrize("name", FACTOR)
def test_golden_residual(oracle, name):
    g = golden(name)
    A, F, T, b = g["A"], g["F"], g["T"], int(g["b"])
    tol = 2e-6 if A.dtype == np.float32 else 1e-14
    assert oracle.residual(A, F, T, b) < tol


def test_structured_tau_two():
    """EYE / upper-triangular inputs: every tau is 2."""
    for prec in ("f32", "f64"):
        for kind in ("eye", "triu"):
            g = golden(f"factor_{prec}_b32_96x96_{kind}.npz")
            T = g["T"]
            for k in range(3):
                assert np.all(T[k * 32, k * 32:] == 2.0)


TILES = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "tile_*.npz")))


@pytest.mark.parametrize("name", TILES)
def test_oracle_tile_bitexact(oracle, name):
    g = golden(name)
    X_in, X_out, tau, b = g["X_in"], g["X_out"], g["tau"], int(g["b"])
    op = name.split("_")[1]
    sfx = oracle.sfx(X_in.dtype)
    L = oracle.L
    X = X_in.copy()
    m = X.shape[1]
    es = X.itemsize
    base = X.ctypes.data
    import ctypes
    P = ctypes.c_void_p
    w = np.zeros(2 * b, X.dtype)
    if op == "geqrt":
        t = np.zeros(b, X.dtype)
        getattr(L, f"oracle_geqrt_{sfx}")(ptr(X), ptr(t), b, b, m, ptr(w))
        assert np.array_equal(t, tau)
    elif op == "unmqr":
        getattr(L, f"oracle_unmqr_{sfx}")(P(base + b * m * es), ptr(X), ptr(tau), b, b, m)
    elif op == "tsqrt":
        t = np.zeros(b, X.dtype)
        getattr(L, f"oracle_tsqrt_{sfx}")(ptr(X), P(base + b * es), ptr(t), b, b, b, m, ptr(w))
        assert np.array_equal(t, tau)
    elif op == "tsmqr":
        getattr(L, f"oracle_tsmqr_{sfx}")(P(base + b * es), P(base + b * m * es), P(base + (b * m + b) * es),
                                          ptr(tau), b, b, m)
    assert np.array_equal(X.view(np.uint8), X_out.view(np.uint8))


@pytest.mark.parametrize("prec,b,m,n", [("f64", 32, 160, 128), ("f32", 32, 128, 160), ("f64", 64, 256, 192),
                                        ("f64", 128, 256, 256), ("f32", 16, 80, 48)])
def test_oracle_vs_reference_build(oracle, prec, b, m, n):
    """Extra shapes straight against oracle/_ref (only where /root/reference was built)."""
    L = ref_lib(("ref_f32" if prec == "f32" else "ref_f64") + ("" if b == 32 else "_fix"))
    if L is None:
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    dt = np.float32 if prec == "f32" else np.float64
    A = oracle.randzo(m, n, dt, seed=7)
    F, T = oracle.factor(A, b)
    F2, T2 = np.zeros_like(A), np.zeros_like(A)
    L.ref_factor(ptr(A), ptr(F2), ptr(T2), m, n, b, m, 4)
    assert np.array_equal(F, F2) and np.array_equal(T, T2)
