"""The reference's legacy entry points (include/gpucalc.h, include/qrdecomp.h) called through
the C ABI on the GPU and checked against the oracle — every declared compute symbol:
cudaQRTask(_d), cudaQRFull, taskQRP_threads(_d), doATask(_d), SGEQRF/SLARFT/STSQRF/SSSRFT and
the D* siblings, testDAPP, doCUDADAPP — plus the wave engine (tqr.h TQR_ENGINE_WAVES) as a
factorisation, and a compiled C driver in the shape of the reference's tiledQR (qrdecomp.c:64-130).

Tolerances: fp64 elementwise <= 1e-11 * max(1, max|F|) (tiles 1e-12), fp32 <= 1e-3 absolute
(the reference's EPSILON, qrdecomp.c:23)."""
import ctypes
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import PKG, REPO

pytestmark = pytest.mark.gpu
P = ctypes.c_void_p


def vp(a, off=0):
    return P(a.ctypes.data + off * a.itemsize)


def tol(dt, scale=1.0):
    return (1e-11 * max(1.0, scale)) if dt == np.float64 else 1e-3


@pytest.mark.parametrize("m,n,b", [(512, 512, 64), (768, 512, 128), (4096, 4096, 128)])
def test_wave_engine_vs_oracle(tqr, oracle, m, n, b):
    """The host-scheduled multi-stream wave engine (BFS waves of the reference DAG, two batched
    launches per wave) reproduces the oracle like the persistent engine does."""
    A = oracle.randzo(m, n, np.float64, seed=5)
    F_ref, T_ref = oracle.factor(A, b, threads=16)
    F = A.copy()
    T = np.zeros_like(A)
    L = tqr.lib()
    assert L.tqr_geqrt_host_engine(1, vp(F), vp(T), m, n, m, b, 0) == 0
    s = float(np.abs(F_ref).max())
    assert float(np.abs(F - F_ref).max()) <= tol(np.float64, s)
    assert float(np.abs(T - T_ref).max()) <= 2e-11


def test_cudaQRFull_and_cudaQRTask_d(tqr, oracle):
    L = tqr.lib()
    m, n = 256, 192
    A = oracle.randzo(m, n, np.float32, seed=5)
    F_ref, _ = oracle.factor(A, 32)
    G = A.copy()
    L.cudaQRFull(vp(G), m, n)
    assert float(np.abs(G - F_ref).max()) <= 1e-3
    Ad = oracle.randzo(m, n, np.float64, seed=7)
    Fd_ref, _ = oracle.factor(Ad, 32)
    Gd = Ad.copy()
    L.cudaQRTask_d(vp(Gd), m, n, m, 128)
    assert float(np.abs(Gd - Fd_ref).max()) <= tol(np.float64, float(np.abs(Fd_ref).max()))


@pytest.mark.parametrize("b", [32, 64])
def test_taskQRP_threads_d(tqr, oracle, b):
    L = tqr.lib()
    m, n = 4 * b, 3 * b
    A = oracle.randzo(m, n, np.float64, seed=3)
    F_ref, T_ref = oracle.factor(A, b)
    R = np.zeros_like(A)
    T = np.zeros_like(A)
    L.taskQRP_threads_d(vp(A), vp(R), vp(T), m, n, b, m, 1)
    assert float(np.abs(R - F_ref).max()) <= tol(np.float64, float(np.abs(F_ref).max()))
    assert float(np.abs(T - T_ref).max()) <= 2e-11


class Task(ctypes.Structure):
    _fields_ = [("taskType", ctypes.c_int), ("l", ctypes.c_int), ("m", ctypes.c_int), ("k", ctypes.c_int),
                ("taskStatus", ctypes.c_int)]


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_doATask_drives_reference_dag(tqr, oracle, dt):
    """Run the whole factorisation as the reference's host runtime does (pthr_doTasks,
    qrdecomp.c:306-361, serialised): getNextTask / doATask / doneATask — every task type goes
    through doATask(_d) on the GPU."""
    L = tqr.lib()
    L.initScheduler.restype = ctypes.POINTER(Task)
    b, M, N = 32, 4, 3
    m, n = M * b, N * b
    A = oracle.randzo(m, n, dt, seed=5)
    F_ref, T_ref = oracle.factor(A, b)
    F = A.copy()
    T = np.zeros_like(A)
    grid = L.initScheduler(M, N)
    fn = L.doATask if dt == np.float32 else L.doATask_d
    fn.argtypes = [Task, P, P, ctypes.c_int, ctypes.c_int, P, ctypes.c_int]
    L.doneATask.argtypes = [ctypes.POINTER(Task), ctypes.c_int, ctypes.c_int, Task]
    L.getNextTask.argtypes = [ctypes.POINTER(Task), ctypes.POINTER(Task), ctypes.c_int, ctypes.c_int]
    seen = set()
    for _ in range(10000):
        t = Task()
        r = L.getNextTask(ctypes.byref(t), grid, M, N)
        if r == 2:
            break
        assert r == 0
        seen.add(t.taskType)
        fn(t, vp(F), vp(T), b, m, None, 1)
        L.doneATask(grid, M, N, t)
    assert seen == {0, 1, 2, 3}
    ctypes.CDLL(None).free(ctypes.cast(grid, P))
    s = float(np.abs(F_ref).max())
    assert float(np.abs(F.astype(np.float64) - F_ref).max()) <= tol(dt, s) * (10 if dt == np.float64 else 1)
    assert float(np.abs(T.astype(np.float64) - T_ref).max()) <= tol(dt, 2.0) * (10 if dt == np.float64 else 1)


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_tile_kernels_by_reference_names(tqr, oracle, dt):
    """SGEQRF/SLARFT/STSQRF/SSSRFT (and DGEQRF/...): the reference's tile kernels by name
    (qrdecomp.h), host pointers into one ldm-strided matrix, against the oracle's tile ops."""
    L = tqr.lib()
    O = oracle.L
    sfx = "S" if dt == np.float32 else "D"
    osfx = "s" if dt == np.float32 else "d"
    b = 32
    m = 2 * b
    M0 = oracle.randzo(m, m, dt, seed=11)   # (n, m) storage: tiles (0,0),(1,0),(0,1),(1,1)
    tl = lambda X, r, c: vp(X, c * b * m + r * b)
    G, R = M0.copy(), M0.copy()
    tg, tr = np.zeros(2 * b, dt), np.zeros(2 * b, dt)
    w = np.zeros(4 * b, dt)
    # GEQRT of tile (0,0)
    getattr(L, f"{sfx}GEQRF")(tl(G, 0, 0), vp(tg), b, b, m, vp(w))
    getattr(O, f"oracle_geqrt_{osfx}")(tl(R, 0, 0), vp(tr), b, b, m, vp(w))
    # UNMQR of tile (0,1) with tile (0,0)'s V
    wp = (P * 2)(vp(w), vp(w, b))
    getattr(L, f"{sfx}LARFT")(tl(G, 0, 1), tl(G, 0, 0), vp(tg), b, b, m, wp)
    getattr(O, f"oracle_unmqr_{osfx}")(tl(R, 0, 1), tl(R, 0, 0), vp(tr), b, b, m)
    # TSQRT of [R(0,0); tile (1,0)]
    getattr(L, f"{sfx}TSQRF")(tl(G, 0, 0), tl(G, 1, 0), vp(tg, b), b, b, b, m, vp(w))
    getattr(O, f"oracle_tsqrt_{osfx}")(tl(R, 0, 0), tl(R, 1, 0), vp(tr, b), b, b, b, m, vp(w))
    # TSMQR of [tile (0,1); tile (1,1)] with tile (1,0)'s V_B
    getattr(L, f"{sfx}SSRFT")(tl(G, 1, 0), tl(G, 0, 1), tl(G, 1, 1), vp(tg, b), b, b, m)
    getattr(O, f"oracle_tsmqr_{osfx}")(tl(R, 1, 0), tl(R, 0, 1), tl(R, 1, 1), vp(tr, b), b, b, m)
    s = float(np.abs(R).max())
    lim = 1e-12 * max(1.0, s) if dt == np.float64 else 1e-4 * max(1.0, s)
    assert float(np.abs(G.astype(np.float64) - R).max()) <= lim
    assert float(np.abs(tg.astype(np.float64) - tr).max()) <= lim


def test_doCUDADAPP(tqr, oracle):
    """One DAPP on a 64 x 64 fp32 matrix with the first 32 entries as taus (gpucalc.cu:1776)."""
    L = tqr.lib()
    X = oracle.randzo(64, 64, np.float32, seed=9)
    ref = X.copy()
    taus = ref.ravel()[:32].copy()
    oracle.L.oracle_tsmqr_s(vp(ref, 32), vp(ref, 32 * 64), vp(ref, 32 * 64 + 32), vp(taus), 32, 32, 64)
    L.doCUDADAPP(vp(X))
    assert float(np.abs(X.astype(np.float64) - ref).max()) <= 1e-4 * max(1.0, float(np.abs(ref).max()))


def test_testDAPP_and_tile_batch(tqr, oracle):
    """testDAPP (gpucalc.cu:1706-1774 semantics): positive timings, ms x nblocks; and the batched
    runner underneath it reproduces the oracle's TSMQR/UNMQR on every copy."""
    L = tqr.lib()
    tm = np.zeros(3, np.float32)
    L.testDAPP(vp(tm), 3, 64)
    assert np.all(np.isfinite(tm)) and np.all(tm > 0)
    for dt, code in ((np.float64, 1), (np.float32, 0)):
        b, nb = 64, 5
        blk = oracle.randzo(2 * b, b, dt, seed=4)          # (b, 2b): [A; B]
        V = oracle.randzo(b, b, dt, seed=6)                 # dense V_B
        tau = (oracle.randzo(b, 1, dt, seed=8).ravel() * 0.5 + 1.5).astype(dt)
        out = np.zeros((nb * b, 2 * b), dt)
        ms = ctypes.c_float()
        assert L.tqr_tile_batch(code, 3, b, nb, vp(V), b, vp(tau), vp(blk), 2 * b, vp(out), 2 * b, ctypes.byref(ms)) == 0
        assert ms.value > 0
        ref = blk.copy()
        Vp = np.zeros((b, 2 * b), dt)  # the oracle's SSSRFT takes one ldm for V, A and B
        Vp[:, :b] = V
        getattr(oracle.L, f"oracle_tsmqr_{oracle.sfx(dt)}")(vp(Vp), vp(ref), vp(ref, b), vp(tau), b, b, 2 * b)
        lim = (1e-12 if dt == np.float64 else 1e-4) * max(1.0, float(np.abs(ref).max()))
        for j in range(nb):
            assert float(np.abs(out[j * b:(j + 1) * b].astype(np.float64) - ref).max()) <= lim


def _build_driver(tmp_path, name):
    gcc = shutil.which("gcc")
    if gcc is None:
        pytest.skip("no gcc")
    exe = str(tmp_path / name)
    subprocess.check_call([gcc, "-O2", "-I" + os.path.join(REPO, "include"),
                           os.path.join(REPO, "tests", "drivers", name + ".c"), "-L" + PKG, "-ltqr",
                           "-Wl,-rpath," + PKG, "-lpthread", "-lm", "-o", exe])
    return exe


def _driver_outputs(path, m, n, count):
    raw = np.fromfile(path, dtype=np.float32)
    assert raw.size == count * m * n
    return [raw[x * m * n:(x + 1) * m * n].reshape(n, m) for x in range(count)]


def test_compiled_c_driver(tmp_path, oracle):
    """INTEGRATION.md's drop-in: a C program in the shape of the reference's tiledQR, built with
    gcc against include/ and libtqr.so, prints "Correct." (its GPU runs agree with each other, the
    reference's own check) — and its outputs match the oracle: taskQRP_threads' matrix and tau and
    cudaQRTask's matrix, elementwise at the reference's EPSILON 1e-3 (qrdecomp.c:23)."""
    exe = _build_driver(tmp_path, "tiledqr_driver")
    out = str(tmp_path / "out.bin")
    r = subprocess.run([exe, "4", out], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Correct." in r.stdout
    m = n = 128
    A, R, T, G = _driver_outputs(out, m, n, 4)
    F_ref, T_ref = oracle.factor(A, 32)
    assert np.abs(R - F_ref).max() <= 1e-3 and np.abs(T - T_ref).max() <= 1e-3
    assert np.abs(G - F_ref).max() <= 1e-3


@pytest.mark.parametrize("threads", [1, 2, 4])
def test_pthr_doTasks_threads(tmp_path, oracle, threads):
    """The reference's worker loop (pthr_doTasks / doPthrBcast, qrdecomp.c:306-367) driven by the
    caller's own pthreads over one task grid (tests/drivers/pthr_driver.c, the thread setup of
    qrdecomp.c:145-230): every task runs on the GPU through doATask; the result matches the oracle
    (fp32, 1e-3 absolute, qrdecomp.c:23) for 1, 2 and 4 threads."""
    exe = _build_driver(tmp_path, "pthr_driver")
    out = str(tmp_path / "out.bin")
    r = subprocess.run([exe, "4", str(threads), out], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout + r.stderr
    m = n = 128
    A, R, T = _driver_outputs(out, m, n, 3)
    F_ref, T_ref = oracle.factor(A, 32)
    assert np.abs(R - F_ref).max() <= 1e-3 and np.abs(T - T_ref).max() <= 1e-3
