"""The C-ABI library loads and exports every function the public headers declare."""
import os
import re

from conftest import REPO


def declared_functions():
    names = set()
    for h in ("tqr.h", "gridscheduler.h", "gpucalc.h", "qrdecomp.h"):
        src = open(os.path.join(REPO, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"typedef[^;]*;", "", src)
        src = re.sub(r"struct\s+\w+\s*\{[^}]*\};", "", src)
        for m in re.finditer(r"\b([A-Za-z_]\w*)\s*\(([^;{]*)\)\s*;", src):
            if m.group(1) not in ("if", "while", "for", "return", "sizeof"):
                names.add(m.group(1))
    return names


def test_exports_all_declared(tqr):
    L = tqr.lib()
    names = declared_functions()
    assert len(names) > 40
    missing = [n for n in sorted(names) if not hasattr(L, n)]
    assert not missing, missing


def test_version_and_errors(tqr):
    L = tqr.lib()
    assert b"gfx950" in L.tqr_version()
    assert L.tqr_strerror(-1) == b"invalid argument"


def test_invalid_args_without_gpu(tqr):
    import ctypes
    L = tqr.lib()
    h = ctypes.c_void_p()
    assert L.tqr_plan_create(ctypes.byref(h), 100, 64, 32, 1) == -1  # b does not divide m
    assert L.tqr_plan_create(ctypes.byref(h), 96, 96, 24, 1) == -1   # unsupported tile size
