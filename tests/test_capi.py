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


def test_leading_dimension_bound_without_gpu(tqr):
    """32 * ldm * sizeof(element) must stay below 2^31 (the engine's 32-bit buffer offsets,
    include/tqr.h): rejected before any device work."""
    import ctypes
    L = tqr.lib()
    h = ctypes.c_void_p()
    m = 8388608 + 256  # > 8,388,607 rows: too tall for fp64
    assert L.tqr_plan_create(ctypes.byref(h), m, 256, 256, 1) == -1
    # the same shape in fp32 passes the bound and only then needs a device (-4 here, no GPU)
    st = L.tqr_plan_create(ctypes.byref(h), m, 256, 256, 0)
    assert st in (-4, 0)
    if st == 0:
        L.tqr_plan_destroy(h)


def test_invalid_engine_and_batch_args_without_gpu(tqr):
    import ctypes
    L = tqr.lib()
    h = ctypes.c_void_p()
    assert L.tqr_plan_create_engine(ctypes.byref(h), 256, 256, 64, 1, 7) == -1
    assert L.tqr_geqrt_host_engine(1, None, None, 256, 256, 256, 64, 0) == -1
    # only the update types (SAPP = 1, DAPP = 3) batch; GEQRT (0) is rejected
    ms = ctypes.c_float()
    assert L.tqr_tile_batch(1, 0, 32, 4, None, 32, None, None, 64, None, 0, ctypes.byref(ms)) == -1
    # a batch beyond the 32-bit offsets of its device matrix (fp64, b = 256: 2049 tiles, 2.15 GB)
    z = ctypes.c_void_p(1)
    assert L.tqr_tile_batch(1, 3, 256, 2048, z, 256, z, z, 512, None, 0, ctypes.byref(ms)) == -1
    assert L.tqr_dist_import(None, None, 0) == -1
    assert L.tqr_plan_execute(None, None, 0, None, None) == -1


def test_flow_plan_export(tqr):
    """The persistent engine's task list (host only): every panel member and chain segment once."""
    import ctypes
    L = tqr.lib()
    M, N = 12, 8
    n = L.tqr_flow_plan_export(M, N, 256, 4, None, 0)
    buf = (ctypes.c_int * (4 * n))()
    assert L.tqr_flow_plan_export(M, N, 256, 4, buf, n) == n
    items = [tuple(buf[4 * x:4 * x + 4]) for x in range(n)]
    panels = [it for it in items if (it[0] & 0xff) != 4]
    assert len(panels) == sum(M - k for k in range(min(M, N)))
    assert len(set(items)) == n


def test_xfer_plan_topological(tqr):
    """The host-API task list (flow list + nxc UP / DOWN tasks per tile column, csrc/xfer.hpp):
    the estimated order is topological for every shape and upload speed, and holds exactly
    2 * q * nxc transfer tasks more than the device-API list."""
    import ctypes
    L = tqr.lib()
    L.tqr_flow_xfer_plan_check.argtypes = [ctypes.c_int] * 5 + [ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p]
    for M, N, nxc, tcol in ((64, 64, 4, 3.4), (256, 64, 16, 13.6), (8, 12, 1, 0.5), (12, 8, 3, 0.0), (1, 1, 1, 1.0)):
        nt0, est0 = ctypes.c_int(), ctypes.c_int()
        assert L.tqr_flow_plan_check(M, N, 256, 8, ctypes.byref(nt0), ctypes.byref(est0)) == 0
        nt, est = ctypes.c_int(), ctypes.c_int()
        assert L.tqr_flow_xfer_plan_check(M, N, 256, 8, nxc, tcol, ctypes.byref(nt), ctypes.byref(est)) == 0
        assert est.value == 1, (M, N)
        assert nt.value == nt0.value + 2 * N * nxc
    assert L.tqr_flow_xfer_plan_check(4, 4, 256, 8, 0, 1.0, None, None) == -1
    assert L.tqr_flow_xfer_plan_check(4, 4, 256, 8, 256, 1.0, None, None) == -1


def step_major(items):
    """A different valid order of a flow list: step by step, panel members first, then the chain
    segments by column, segment, strip (the engine's always-topological fallback order)."""
    def key(it):
        ty = it[0] & 0xff
        if ty == 4:
            return (it[3] & 0xffff, 1, it[2], it[3] >> 16, (it[0] >> 8) & 0xff)
        return (it[3], 0, it[1], 0, 0)
    return sorted(items, key=key)


def test_order_check_accepts_valid_rejects_invalid(tqr):
    """tqr_flow_order_check (the condition tqr_plan_set_tasks enforces): the exported order and a
    step-major permutation are accepted; a chain segment moved in front of its panel, or a
    dropped task, is rejected."""
    import ctypes
    L = tqr.lib()
    M, N, b = 10, 6, 256
    n = L.tqr_flow_plan_export(M, N, b, 4, None, 0)
    buf = (ctypes.c_int * (4 * n))()
    L.tqr_flow_plan_export(M, N, b, 4, buf, n)
    items = [tuple(buf[4 * x:4 * x + 4]) for x in range(n)]

    def check(lst):
        arr = (ctypes.c_int * (4 * len(lst)))(*[v for it in lst for v in it])
        return L.tqr_flow_order_check(M, N, b, arr, len(lst))

    assert check(items) == 1
    sm = step_major(items)
    assert sm != items and check(sm) == 1
    first_chain = next(x for x, it in enumerate(sm) if (it[0] & 0xff) == 4)
    bad = [sm[first_chain]] + sm[:first_chain] + sm[first_chain + 1:]
    assert check(bad) == 0
    assert check(sm[1:]) == 0  # GEQRT(0) missing: everything waits on it
