"""Host-pointer API with the transfers inside the persistent launch (csrc/xfer.hpp): the launch
reads each tile column from host memory before step 0 needs it and writes it back once final.
Checked against the oracle (the reference host path restated; SURVEY.md §8d tolerances) for both
host-memory modes (pinned staging filled / drained by host threads while the kernel runs, and the
caller's array registered), strided and odd leading dimensions (16-B and element paths), fp32,
wide and tall shapes, tau discarded, and repeated calls on one staging buffer."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _strided(A, ldm):
    """copy of A (n, m) into an (n, ldm) array whose rows m.. hold a sentinel"""
    n, m = A.shape
    S = np.full((n, ldm), 7.25, dtype=A.dtype)
    S[:, :m] = A
    return S


def _check(F, T, F_ref, T_ref):
    if F_ref.dtype == np.float64:
        assert np.abs(F - F_ref).max() <= 1e-11 * max(1.0, np.abs(F_ref).max())
        if T is not None:
            assert np.abs(T - T_ref).max() <= 2e-11
    else:
        assert np.abs(F.astype(np.float64) - F_ref).max() <= 1e-3
        if T is not None:
            assert np.abs(T.astype(np.float64) - T_ref).max() <= 1e-3


@pytest.fixture(params=["stage", "register"])
def mode(request):
    old = os.environ.get("TQR_HOST_XFER")
    os.environ["TQR_HOST_XFER"] = request.param
    yield request.param
    if old is None:
        os.environ.pop("TQR_HOST_XFER", None)
    else:
        os.environ["TQR_HOST_XFER"] = old


@pytest.mark.parametrize("m,n,b,dt,pad", [
    (1024, 768, 128, np.float64, 16),   # strided, 16-B path
    (512, 512, 64, np.float64, 1),      # odd ldm: element path
    (768, 1024, 128, np.float64, 0),    # wide
    (2048, 512, 256, np.float64, 0),    # tall: several chunks per column
    (512, 512, 64, np.float32, 4),
    (1024, 1024, 256, np.float32, 3),   # fp32, unaligned columns
])
def test_host_xfer_vs_oracle(tqr, oracle, mode, m, n, b, dt, pad):
    A = oracle.randzo(m, n, dt, seed=11)
    F_ref, T_ref = oracle.factor(A, b, threads=8)
    F = _strided(A, m + pad)
    T = tqr.geqrt_host(F, b, m=m)
    _check(F[:, :m], T[:, :m], F_ref, T_ref)
    assert np.all(F[:, m:] == 7.25) and np.all(T[:, m:] == 0)  # rows beyond m untouched


def test_host_xfer_no_tau_and_repeats(tqr, oracle):
    """tau discarded (cudaQRTask's contract), three calls in a row on one staging buffer (the
    flag generation advances), then a larger shape (the staging buffer grows)."""
    m, n, b = 1024, 1024, 128
    A = oracle.randzo(m, n, np.float64, seed=3)
    F_ref, T_ref = oracle.factor(A, b, threads=8)
    for _ in range(3):
        F = A.copy()
        assert tqr.geqrt_host(F, b, with_tau=False) is None
        _check(F, None, F_ref, None)
    A2 = oracle.randzo(2048, 1024, np.float64, seed=4)
    F2_ref, T2_ref = oracle.factor(A2, b, threads=8)
    F2 = A2.copy()
    T2 = tqr.geqrt_host(F2, b)
    _check(F2, T2, F2_ref, T2_ref)


def test_cache_clear_then_reuse(tqr, oracle):
    m = n = 512
    b = 64
    A = oracle.randzo(m, n, np.float64, seed=5)
    F_ref, T_ref = oracle.factor(A, b)
    F = A.copy()
    tqr.geqrt_host(F, b)
    tqr.cache_clear()
    F = A.copy()
    T = tqr.geqrt_host(F, b)
    _check(F, T, F_ref, T_ref)


def test_slow_host_staging_beyond_the_kernel_wait_limit(tqr, oracle):
    """A host that stages the input slower than the engine's 5 s wait limit (one host
    thread on a 32 GiB matrix): every tile column is staged 800 ms late (TQR_HOST_STAGE_DELAY_MS,
    8 columns: 6.4 s). A wait that expires re-arms whenever the launch's upload count has moved
    since its previous expiry (flow.hpp timed_out: progress-based), so the launch waits for as
    long as the host keeps staging and completes."""
    m, n, b = 512, 2048, 256
    A = oracle.randzo(m, n, np.float64, seed=9)
    F_ref, T_ref = oracle.factor(A, b)
    os.environ["TQR_HOST_STAGE_DELAY_MS"] = "800"
    try:
        F = A.copy()
        T = tqr.geqrt_host(F, b)
    finally:
        os.environ.pop("TQR_HOST_STAGE_DELAY_MS", None)
    _check(F, T, F_ref, T_ref)


def test_cache_clear_concurrent_with_calls(tqr, oracle):
    """tqr_cache_clear while other threads run one-shot host-API calls on cached plans:
    no call may use a freed plan or staging buffer, and every result stays exact."""
    import threading
    m = n = 512
    b = 64
    A = oracle.randzo(m, n, np.float64, seed=6)
    F_ref, T_ref = oracle.factor(A, b)
    errs = []

    def worker():
        try:
            for _ in range(4):
                F = A.copy()
                T = tqr.geqrt_host(F, b)
                _check(F, T, F_ref, T_ref)
        except Exception as e:  # noqa: BLE001 (reported below)
            errs.append(e)

    th = [threading.Thread(target=worker) for _ in range(2)]
    for t in th:
        t.start()
    for _ in range(6):
        tqr.cache_clear()
    for t in th:
        t.join()
    assert not errs, errs
