"""The product scheduler (csrc/sched.c) against the reference scheduler's own behaviour."""
import numpy as np
import pytest

from conftest import golden


def test_trace_matches_reference(tqr):
    g = golden("sched.npz")
    for key in g.files:
        if not key.startswith("trace_"):
            continue
        M, N = map(int, key.split("_")[1].split("x"))
        s = tqr.Scheduler(M, N)
        out = []
        while True:
            r, t = s.next_task()
            if r != tqr.TASK_AVAIL:
                assert r == tqr.TASK_DONE
                break
            out.append((t.taskType, t.l, t.m, t.k))
            s.done(t)
        assert np.array_equal(np.array(out, dtype=np.int32).reshape(-1, 4), g[key]), key


def test_waves_match_reference(tqr):
    g = golden("sched.npz")
    for key in g.files:
        if not key.startswith("levels_"):
            continue
        M, N = map(int, key.split("_")[1].split("x"))
        waves = tqr.sched_plan(M, N)
        assert np.array_equal(np.array([len(w) for w in waves]), g[key]), key


@pytest.mark.parametrize("M,N", [(1, 1), (5, 3), (3, 5), (7, 7), (64, 64), (256, 64)])
def test_plan_is_topological(tqr, M, N):
    """Every dependency of a task sits in an earlier wave; every task appears once; inside a
    wave no two tasks write the same tile."""
    waves = tqr.sched_plan(M, N)
    wave_of = {}
    for L, w in enumerate(waves):
        for (ty, l, m, k) in w:
            assert (l, m, k) not in wave_of
            wave_of[(l, m, k)] = L
    assert len(wave_of) == tqr.lib().tqr_sched_total_tasks(M, N)
    for (l, m, k), L in wave_of.items():
        deps = []
        if k > 0:
            deps.append((l, m, k - 1))
        if l == k and m > k:
            deps.append((k, k, k))
        if l > k and m == k:
            deps.append((l - 1, k, k))
        if l > k and m > k:
            deps += [(l, k, k), (l - 1, m, k)]
        for d in deps:
            assert wave_of[d] < L
        if M * N <= 49:
            continue
    for w in waves:  # writes inside a wave are disjoint
        written = set()
        for (ty, l, m, k) in w:
            tiles = {(l, m)} | ({(k, m)} if ty == tqr.DAPP else set()) | ({(k, k)} if ty == tqr.QRD else set())
            assert not (tiles & written)
            written |= tiles


def test_total_tasks(tqr):
    assert tqr.lib().tqr_sched_total_tasks(64, 64) == 89440
    assert tqr.lib().tqr_sched_total_tasks(256, 64) == 488800
    assert tqr.lib().tqr_sched_total_tasks(3, 6) == 32  # the reference's calcTotalTasks says 28
    assert tqr.lib().tqr_total_tasks(16384, 16384, 256) == 89440
    assert tqr.lib().tqr_total_tasks(100, 64, 32) == -1


@pytest.mark.parametrize("M,N,b,seg", [(64, 64, 256, 8), (32, 32, 128, 8), (8, 8, 64, 8), (256, 64, 256, 8),
                                       (3, 6, 32, 2), (6, 3, 32, 2), (1, 1, 32, 8), (5, 7, 16, 1), (1, 5, 32, 4)])
def test_flow_plan_topological(tqr, M, N, b, seg):
    """The persistent engine's task list (panel tasks + chain segments) is in an order where
    every task waits only on earlier tasks — the engine's deadlock-freedom condition."""
    import ctypes
    n, o = ctypes.c_int(), ctypes.c_int()
    assert tqr.lib().tqr_flow_plan_check(M, N, b, seg, ctypes.byref(n), ctypes.byref(o)) == 0
    kmax = min(M, N)
    sw = tqr.lib().tqr_flow_strip_width()
    assert sw in (64, 128)
    ns = (b + sw - 1) // sw
    panels = sum(M - k for k in range(kmax))
    # fp64 list: the last `tail` steps (columns with <= 31 rows below the diagonal) run one-element
    # segments (engine.hip default_tail)
    tail = max(0, min(kmax, kmax - (M - 1 - 31)))
    sl = lambda k: 1 if k >= kmax - tail else seg
    chains = sum((N - k - 1) * ns * max(1, -(-(M - k - 1) // sl(k))) for k in range(kmax))
    # ... and their lookahead column's UNMQR element in a segment of its own (flow.hpp unmqr_alone)
    chains += sum(ns for k in range(kmax) if k >= kmax - tail and M - k - 1 > 0 and k + 1 < N)
    assert n.value == panels + chains
    assert o.value == 1


@pytest.mark.parametrize("M,N,b", [(8, 8, 64), (8, 8, 128), (64, 64, 256), (16, 6, 256), (6, 16, 256)])
def test_flow_plan_segments_below_diagonal(tqr, M, N, b):
    """Every chain segment's rows lie strictly below its step's diagonal tile and segments of one
    chain tile its rows exactly once (the lookahead column's UNMQR-only segment has none): the
    kernel's element loop starts at the UNMQR (segment 0) and runs rows i0 .. i1-1."""
    import ctypes
    cap = 4 * 100000
    buf = (ctypes.c_int * cap)()
    n = tqr.lib().tqr_flow_plan_export(M, N, b, 8, buf, cap)
    assert 0 < n <= cap // 4
    rows = {}
    for x in range(n):
        ts, l, m, k = buf[4 * x:4 * x + 4]
        if ts & 0xff != 4:
            continue
        kk, e, i0, i1, s = k & 0xffff, k >> 16, l & 0xffff, l >> 16, (ts >> 8) & 0xff
        assert kk + 1 <= i0 <= i1 <= M, (kk, m, e, i0, i1)
        rows.setdefault((kk, m, s), []).append((e, i0, i1))
    for (kk, j, s), segs in rows.items():
        segs.sort()
        assert [e for e, _, _ in segs] == list(range(len(segs)))
        covered = [i for _, i0, i1 in segs for i in range(i0, i1)]
        assert covered == list(range(kk + 1, M)), (kk, j, segs)
