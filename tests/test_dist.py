"""Multi-GPU path (tile-column snake partition).

CPU (no GPU): every rank's task list is the global list restricted to its tile columns plus
one forward task per owned panel member — checked for world sizes 1-8 and inside a world-2
gloo process group (as the bench's ranks build them).
GPU: two or four ranks on ONE device (the box has one GPU), each with a share of the CUs, run the
real protocol — IPC-opened peer workspaces, forward tasks, uncached member flags — and must
reproduce the single-GPU engine bit for bit (the per-tile operation sequence is the same).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "gpu-tiled-qr-decomposition_amd"))
import tqr  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _global_list_len(M, N, b, world, monkeypatch):
    """Tasks of the global list a plan of `world` whole-device ranks builds (engine.hip
    multi_rank_defaults: 4+ ranks get one-element segments in the last 7/16 of the steps and the
    lookahead column keyed 4 elements earlier; no rank's list has lone UNMQR segments)."""
    kmax = min(M, N)
    with monkeypatch.context() as mp:
        if world >= 4:
            tail = max(max(0, min(kmax, kmax - (M - 1 - 31))), 7 * kmax // 16)  # (default_tail)
            mp.setenv("TQR_TAIL", str(max(0, tail)))
            mp.setenv("TQR_TAIL_SEGLEN", "1")
            mp.setenv("TQR_LAC", "4")
        if world > 1:
            mp.setenv("TQR_UNMQR_ALONE", "0")
        return tqr.lib().tqr_flow_plan_export(M, N, b, 8, None, 0)


@pytest.mark.parametrize("M,N", [(8, 8), (16, 4), (5, 7), (64, 64)])
def test_partition_covers_global_list(M, N, monkeypatch):
    b = 256
    kmax = min(M, N)
    npanel = sum(M - k for k in range(kmax))
    assert tqr.dist_plan_check(M, N, b, 0, 1)[0] == _global_list_len(M, N, b, 1, monkeypatch)
    for world in (2, 3, 4, 8):
        total = _global_list_len(M, N, b, world, monkeypatch)
        tasks = fwd = 0
        for r in range(world):
            nt, nf = tqr.dist_plan_check(M, N, b, r, world)
            tasks += nt
            fwd += nf
            own_panel = sum(M - k for k in range(kmax) if tqr.tile_owner(k, world) == r)
            assert nf == own_panel
        assert fwd == npanel
        assert tasks == total  # panel tasks forward their own images: no extra tasks


@pytest.mark.parametrize("q,world", [(64, 8), (64, 4), (16, 2), (24, 8)])
def test_snake_partition_balances_column_work(q, world):
    """Every rank owns q/world tile columns whose indices sum to the same total (the chain work of
    column j grows with j); the round-2 cyclic j % world gave the last rank the most."""
    cols = [tqr.owned_tile_cols(q, r, world) for r in range(world)]
    assert sorted(c for cs in cols for c in cs) == list(range(q))
    assert {len(cs) for cs in cols} == {q // world}
    if (q // world) % 2 == 0:
        assert len({sum(cs) for cs in cols}) == 1


def test_cyclic_partition_knob(monkeypatch):
    """TQR_DIST_PART=cyclic (A/B diagnostics) switches the library and tqr.tile_owner together."""
    monkeypatch.setenv("TQR_DIST_PART", "cyclic")
    M, N, world = 16, 8, 4
    for r in range(world):
        assert tqr.owned_tile_cols(N, r, world) == list(range(r, N, world))
        _, nf = tqr.dist_plan_check(M, N, 256, r, world)
        assert nf == sum(M - k for k in range(N) if k % world == r)


def _gloo_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    nt, nf = tqr.dist_plan_check(32, 16, 256, rank, world)
    import torch
    t = torch.tensor([nt, nf], dtype=torch.long)
    dist.all_reduce(t)
    q.put((rank, int(t[0]), int(t[1])))
    dist.destroy_process_group()


def test_partition_gloo_world2(monkeypatch):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    total = _global_list_len(32, 16, 256, 2, monkeypatch)
    npanel = sum(32 - k for k in range(16))
    for _, nt, nf in res:
        assert nf == npanel and nt == total


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("m,n,b,dt,ranks,mode,extra", [(1024, 1024, 128, "f64", 2, "gather", {}), (2048, 768, 256, "f64", 2, "gather", {}),
                                                       (512, 1024, 64, "f64", 2, "gather", {}), (1024, 512, 128, "f32", 2, "gather", {}),
                                                       (2048, 2048, 256, "f64", 4, "gather", {}),
                                                       # the 8-GPU default segment length (2) against one GPU's (8)
                                                       (2048, 2048, 256, "f64", 4, "gather", {"TQR_SEGLEN": "2", "TQR_TEST_REF_SEGLEN": "8"}),
                                                       # ... and the rest of the 8-GPU defaults: one-element segments in the last
                                                       # 7/16 of the steps with the lookahead column keyed 4 elements earlier
                                                       (2048, 2048, 256, "f64", 4, "gather", {"TQR_SEGLEN": "2", "TQR_TAIL": "3",
                                                                                              "TQR_TAIL_SEGLEN": "1", "TQR_LAC": "4",
                                                                                              "TQR_TEST_REF_SEGLEN": "8"}),
                                                       # BASELINE configs[3] shape at full size
                                                       (65536, 16384, 256, "f64", 2, "checksum", {})])
def test_ranks_on_one_gpu_match_single_gpu(m, n, b, dt, ranks, mode, extra):
    env = dict(os.environ, TQR_FLOW_GRID=str(192 // ranks), **extra)
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.join(HERE, "dist_worker.py"), str(m), str(n), str(b), dt, "0", mode]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=500)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    for run in ("run0", "run1"):
        assert res[run]["cols_covered"]
        # same tile operations in the same order on every rank: bit-identical to one GPU
        assert res[run]["exact"], res[run]


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_rank_launching_late_is_waited_for():
    """One rank starts its factorisations 8 s after its peer (longer than the single-GPU 5 s wait
    limit): the peer's waits on its flags outlast the skew (multi-GPU limit 60 s) and both launches
    still match one GPU bit for bit."""
    env = dict(os.environ, TQR_FLOW_GRID="96", TQR_TEST_SKEW_S="8")
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.join(HERE, "dist_worker.py"), "1024", "1024", "128", "f64", "0", "gather"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    for run in ("run0", "run1"):
        assert res[run]["exact"], res[run]


class _ProbeLib:
    """tqr_dist_probe stand-in: phase 1 reports the peers in `seen` (bit mask) and fails if any is
    missing, as the library does."""

    def __init__(self, world, seen):
        self.world, self.seen, self.calls = world, seen, []

    def tqr_dist_probe(self, h, phase, out):
        self.calls.append(phase)
        if phase == 1:
            out._obj.value = self.seen
            return 0 if self.seen == ((1 << self.world) - 1) & ~1 else -3
        return 0

    def tqr_strerror(self, st):
        return b"HIP runtime call failed"


def test_peer_probe_reports_missing_ranks():
    """CPU mock of the setup probe: rank 0 of 4 sees ranks 1 and 3 but not 2 -> the error names
    rank 2 and says why, after put, barrier, check in that order."""
    L = _ProbeLib(4, 0b1010)
    order = []
    with pytest.raises(tqr.TQRError, match=r"rank 0 does not see the flag stores of rank\(s\) \[2\]"):
        tqr.peer_probe(L, None, 0, 4, lambda: order.append("barrier"))
    assert L.calls == [0, 1] and order == ["barrier"]


def test_peer_probe_passes_when_every_peer_is_seen():
    L = _ProbeLib(4, 0b1110)
    assert tqr.peer_probe(L, None, 0, 4, lambda: None) == 0b1110


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_ranks_with_different_task_lists_fail_at_import():
    """A rank whose task list differs (here its chain segment length) would deadlock the launch:
    tqr_dist_import compares the ranks' list signatures and both ranks fail cleanly instead."""
    env = dict(os.environ, TQR_FLOW_GRID="96", TQR_TEST_SEGLEN_RANK1="4")
    env.pop("TQR_SEGLEN", None)
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.join(HERE, "dist_worker.py"), "1024", "1024", "128", "f64", "0", "gather"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode != 0
    assert "built different task lists" in r.stderr, r.stderr[-2000:]
