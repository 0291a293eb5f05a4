"""Shared fixtures: loaders for the oracle (test infrastructure only) and the product lib."""
import ctypes
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "gpu-tiled-qr-decomposition_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, PKG)
sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")


P = ctypes.c_void_p


def ptr(a):
    return a.ctypes.data_as(P)


class Oracle:
    """ctypes view of oracle/liboracle.so (the checker, never the thing measured)."""

    def __init__(self):
        path = os.path.join(REPO, "oracle", "liboracle.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle"), "liboracle.so"])
        self.L = ctypes.CDLL(path)
        self.L.oracle_residual_d.restype = ctypes.c_double

    def sfx(self, dt):
        return "d" if np.dtype(dt) == np.float64 else "s"

    def randzo(self, m, n, dt, seed=5):
        A = np.zeros((n, m), dtype=dt)
        getattr(self.L, f"oracle_randzo_{self.sfx(dt)}")(ptr(A), m, n, m, seed)
        return A

    def factor(self, A, b, threads=0):
        n, m = A.shape
        F = np.zeros_like(A)
        T = np.zeros_like(A)
        if threads:
            getattr(self.L, f"oracle_factor_threads_{self.sfx(A.dtype)}")(ptr(A), ptr(F), ptr(T), m, n, b, m, threads)
        else:
            getattr(self.L, f"oracle_factor_serial_{self.sfx(A.dtype)}")(ptr(A), ptr(F), ptr(T), m, n, b, m)
        return F, T

    def residual(self, A, F, T, b):
        n, m = A.shape
        a, f, t = (np.ascontiguousarray(x, dtype=np.float64) for x in (A, F, T))
        return self.L.oracle_residual_d(ptr(a), ptr(f), ptr(t), m, n, b, m)


@pytest.fixture(scope="session")
def oracle():
    return Oracle()


@pytest.fixture(scope="session")
def tqr():
    import tqr as mod
    return mod


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def ref_lib(name):
    """oracle/_ref/lib<name>.so if it was built here (it needs /root/reference)."""
    path = os.path.join(REPO, "oracle", "_ref", f"lib{name}.so")
    if not os.path.exists(path):
        return None
    L = ctypes.CDLL(path)
    L.ref_factor.restype = ctypes.c_double
    return L


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
