"""Generate the golden fixtures in tests/golden/ from the reference's own host code.

Runs here only (needs /root/reference, via oracle/_ref/ built by oracle/build_ref.sh).
Every fixture is data — inputs and the reference's outputs — never reference source:

  factor_<prec>_b<b>_<m>x<n>_<input>.npz   A (input), F (in-place R+V), T (m x n tau matrix)
  tile_<op>_<prec>_b<b>.npz                single-tile known answers for SGEQRF/SLARFT/STSQRF/SSSRFT
  sched.npz                                scheduler traces and BFS wave sizes

Arrays are stored column-major as numpy arrays of shape (n, m) (row j = column j of the
matrix), exactly the reference's CO(i,j,ldm) = j*ldm + i layout with ldm = m.
Inputs: RANDZO after srand(seed) (qrdecomp.c:81,89,1383), EYE (qrdecomp.c:1385) and an
upper-triangular RANDZO matrix (tau = 2 everywhere).
"""
import ctypes
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REFDIR = os.path.join(REPO, "oracle", "_ref")
P = ctypes.c_void_p


def ptr(a):
    return a.ctypes.data_as(P)


def load(name):
    lib = ctypes.CDLL(os.path.join(REFDIR, f"lib{name}.so"))
    lib.ref_factor.restype = ctypes.c_double
    return lib


def refname(prec, b):
    # b == 32: the reference exactly as shipped; else the one-line qrdecomp.c:506 fix.
    return ("ref_f32" if prec == "f32" else "ref_f64") + ("" if b == 32 else "_fix")


def make_input(lib, dt, m, n, kind, seed):
    A = np.zeros((n, m), dtype=dt)
    if kind == "randzo":
        lib.ref_randzo(ptr(A), m, n, m, seed)
    elif kind == "eye":
        for i in range(min(m, n)):
            A[i, i] = 1
    elif kind == "triu":
        lib.ref_randzo(ptr(A), m, n, m, seed)
        for j in range(n):
            A[j, j + 1:] = 0
    return A


def factor_case(prec, b, m, n, kind, seed=5):
    dt = np.float32 if prec == "f32" else np.float64
    lib = load(refname(prec, b))
    A = make_input(lib, dt, m, n, kind, seed)
    F = np.zeros_like(A)
    T = np.zeros_like(A)
    lib.ref_factor(ptr(A), ptr(F), ptr(T), m, n, b, m, 8)
    name = f"factor_{prec}_b{b}_{m}x{n}_{kind}.npz"
    np.savez_compressed(os.path.join(HERE, name), A=A, F=F, T=T, m=m, n=n, b=b, seed=seed)
    return name


def tile_cases(prec, b):
    """One known-answer vector per tile kernel, on one 2b x 2b RANDZO block (seed 11)."""
    dt = np.float32 if prec == "f32" else np.float64
    lib = load(refname(prec, b))
    m = 2 * b
    A = np.zeros((m, m), dtype=dt)
    lib.ref_randzo(ptr(A), m, m, m, 11)
    names = []
    # GEQRT on tile (0,0)
    X = A.copy(); tau = np.zeros(b, dt)
    lib.ref_geqrt(ptr(X), ptr(tau), b, m)
    names.append(_save_tile("geqrt", prec, b, A, X, tau))
    geq, geq_tau = X.copy(), tau.copy()
    # UNMQR: C = tile (0,1) with V/tau of the GEQRT above
    X = geq.copy()
    lib.ref_unmqr(ctypes.c_void_p(X.ctypes.data + b * m * X.itemsize), ptr(X), ptr(geq_tau), b, m)
    names.append(_save_tile("unmqr", prec, b, geq, X, geq_tau))
    # TSQRT: A = R of tile (0,0), B = tile (1,0)
    X = geq.copy(); tau = np.zeros(b, dt)
    lib.ref_tsqrt(ptr(X), ctypes.c_void_p(X.ctypes.data + b * X.itemsize), ptr(tau), b, m)
    names.append(_save_tile("tsqrt", prec, b, geq, X, tau))
    tsq, tsq_tau = X.copy(), tau.copy()
    # TSMQR: V = tile (1,0), A = tile (0,1), B = tile (1,1)
    X = tsq.copy()
    base, es = X.ctypes.data, X.itemsize
    lib.ref_tsmqr(ctypes.c_void_p(base + b * es), ctypes.c_void_p(base + b * m * es),
                  ctypes.c_void_p(base + (b * m + b) * es), ptr(tsq_tau), b, m)
    names.append(_save_tile("tsmqr", prec, b, tsq, X, tsq_tau))
    return names


def _save_tile(op, prec, b, X_in, X_out, tau):
    name = f"tile_{op}_{prec}_b{b}.npz"
    np.savez_compressed(os.path.join(HERE, name), X_in=X_in, X_out=X_out, tau=tau, b=b)
    return name


def sched_cases():
    lib = load("ref_f64")
    out = {}
    for (M, N) in [(1, 1), (2, 2), (3, 2), (2, 3), (4, 4), (3, 6), (8, 8)]:
        cap = M * N * min(M, N) + 8
        buf = np.zeros(4 * cap, dtype=np.int32)
        cnt = lib.ref_sched_trace(M, N, ptr(buf), cap)
        out[f"trace_{M}x{N}"] = buf[: 4 * cnt].reshape(cnt, 4)
    for (M, N) in [(8, 8), (32, 32), (64, 64), (256, 64), (3, 6), (6, 3)]:
        lv = np.zeros(4096, dtype=np.int32)
        L = lib.ref_sched_levels(M, N, ptr(lv), 4096)
        out[f"levels_{M}x{N}"] = lv[:L].copy()
    np.savez_compressed(os.path.join(HERE, "sched.npz"), **out)
    return "sched.npz"


def main():
    if not os.path.exists(os.path.join(REFDIR, "libref_f64.so")):
        sys.exit("oracle/_ref not built (run oracle/build_ref.sh here, where /root/reference exists)")
    names = []
    for prec in ("f32", "f64"):
        for (m, n) in [(64, 64), (96, 64), (64, 96)]:
            names.append(factor_case(prec, 32, m, n, "randzo"))
        names.append(factor_case(prec, 32, 96, 96, "eye"))
        names.append(factor_case(prec, 32, 96, 96, "triu"))
        names.append(factor_case(prec, 16, 64, 48, "randzo"))
        names += tile_cases(prec, 32)
    names.append(factor_case("f64", 64, 128, 128, "randzo"))
    names.append(factor_case("f64", 64, 192, 128, "randzo"))
    names += tile_cases("f64", 64)
    names.append(sched_cases())
    with open(os.path.join(HERE, "MANIFEST.md5"), "w") as f:
        for nm in sorted(names):
            h = hashlib.md5(open(os.path.join(HERE, nm), "rb").read()).hexdigest()
            f.write(f"{h}  {nm}\n")
    total = sum(os.path.getsize(os.path.join(HERE, nm)) for nm in names)
    print(f"wrote {len(names)} fixtures, {total / 1024:.0f} KiB")


if __name__ == "__main__":
    main()
