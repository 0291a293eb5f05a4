"""CPU tests of bench.py's output checks (run outside the timed region of every bench line):
the single-GPU column-norm check and the per-rank check of a multi-GPU factorisation."""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def _factored(m, n, seed=3):
    """A (n, m)-stored matrix and a factorisation in the engine's layout: R in the upper triangle,
    arbitrary values below it (the engine keeps V there)."""
    g = torch.Generator().manual_seed(seed)
    M = torch.randn(m, n, dtype=torch.float64, generator=g)
    _, R = torch.linalg.qr(M)
    F = torch.randn(m, n, dtype=torch.float64, generator=g)
    F[:n] = torch.triu(R) + torch.tril(F[:n], -1)
    return M.T.contiguous(), F.T.contiguous()


def test_check_output_accepts_and_rejects():
    A0, A = _factored(256, 128)
    assert bench.check_output(A0, A, 256, 128) < 1e-12
    A[5, 2] += 1.0  # an R entry (row 2 <= column 5)
    with pytest.raises(RuntimeError):
        bench.check_output(A0, A, 256, 128)


@pytest.mark.parametrize("world", [1, 2, 4])
def test_check_owned_columns_every_rank(world):
    m, n, b = 256, 128, 16
    A0, A = _factored(m, n)
    for rank in range(world):
        assert bench.check_owned_columns(A0, A, m, n, b, rank, world) < 1e-12


def test_check_owned_columns_sees_only_its_columns():
    m, n, b = 256, 128, 16
    A0, A = _factored(m, n)
    A[b + 3, 7] += 1.0  # column b+3: tile column 1 -> rank 1 of 2
    assert bench.check_owned_columns(A0, A, m, n, b, 0, 2) < 1e-12
    with pytest.raises(RuntimeError):
        bench.check_owned_columns(A0, A, m, n, b, 1, 2)
    A[b + 3, 7] -= 1.0
    A[b + 3, 200] += 1.0  # below the diagonal (V): not part of R
    assert bench.check_owned_columns(A0, A, m, n, b, 1, 2) < 1e-12


# ---- bench.py --gpus N launch decision (a plain `bench.py --gpus N` must start N ranks) ----
def _ndev(n):
    def f():
        return n
    return f


def test_launch_plan_decisions():
    assert bench.launch_plan(1, {}, _ndev(8)) == ("run", None)
    assert bench.launch_plan(8, {}, _ndev(8)) == ("spawn", None)
    how, msg = bench.launch_plan(8, {}, _ndev(4))
    assert how == "error" and "only 4" in msg
    # one-GPU rehearsal: every rank pinned to one device, the device count does not bound N
    assert bench.launch_plan(4, {"TQR_BENCH_DEVICE": "0"}, _ndev(1)) == ("spawn", None)
    # under an external launcher: run as one of its ranks, and --gpus must agree with it
    assert bench.launch_plan(2, {"WORLD_SIZE": "2"}, _ndev(0)) == ("run", None)
    how, msg = bench.launch_plan(4, {"WORLD_SIZE": "2"}, _ndev(8))
    assert how == "error" and "WORLD_SIZE" in msg
    assert bench.launch_plan(0, {}, _ndev(8))[0] == "error"


def test_launch_plan_does_not_count_devices_unless_needed():
    def boom():
        raise AssertionError("device count asked")
    assert bench.launch_plan(1, {}, boom) == ("run", None)
    assert bench.launch_plan(2, {"WORLD_SIZE": "2"}, boom) == ("run", None)
    assert bench.launch_plan(2, {"TQR_BENCH_DEVICE": "0"}, boom) == ("spawn", None)


class _FakeChild:
    def __init__(self, lines, rc):
        self.stdout = iter(lines)
        self._rc = rc

    def wait(self):
        return self._rc


def test_spawn_ranks_relays_json_and_exit_code(capsys):
    seen = {}

    def popen(cmd, **kw):
        seen["cmd"] = cmd
        return _FakeChild(["noise from a rank\n", '{"metric": "m", "value": 1.0, "n_gpus": 2}\n'], 0)

    rc = bench.spawn_ranks(2, ["--gpus", "2", "--steps", "3"], popen=popen)
    out, err = capsys.readouterr()
    assert rc == 0
    assert out.strip() == '{"metric": "m", "value": 1.0, "n_gpus": 2}'
    assert "noise from a rank" in err
    cmd = seen["cmd"]
    assert cmd[1:4] == ["-u", "-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "2", "--steps", "3"] and cmd[-5].endswith("bench.py")


def test_spawn_ranks_failure_modes(capsys):
    assert bench.spawn_ranks(2, [], popen=lambda cmd, **kw: _FakeChild(["x\n"], 0)) == 1  # no result line
    assert bench.spawn_ranks(2, [], popen=lambda cmd, **kw: _FakeChild([], 3)) == 3  # the child's code
    capsys.readouterr()


@pytest.mark.parametrize("world", [2, 4])
def test_check_owned_columns_packed_storage(world):
    """The multi-GPU storage: a rank holds only its own tile columns, packed in column order."""
    import tqr
    m, n, b = 256, 128, 16
    A0, A = _factored(m, n)
    for rank in range(world):
        own = tqr.owned_tile_cols(n // b, rank, world)
        rows = torch.cat([torch.arange(j * b, (j + 1) * b) for j in own])
        assert bench.check_owned_columns(A0[rows], A[rows], m, n, b, rank, world, own, packed=True) < 1e-12
        Ab = A[rows].clone()
        Ab[b + 3, 0] += 1.0  # an R entry of the rank's second tile column (row 0 <= its column)
        with pytest.raises(RuntimeError):
            bench.check_owned_columns(A0[rows], Ab, m, n, b, rank, world, own, packed=True)


def test_chain_segment_length_rule(monkeypatch):
    """bench.seglen_of mirrors engine.hip env_seglen: 8 on one or two ranks, 2 from four ranks on
    (tools/sched_sim.py seglen), TQR_SEGLEN overrides."""
    monkeypatch.delenv("TQR_SEGLEN", raising=False)
    assert [bench.seglen_of(w) for w in (1, 2, 4, 8)] == [8, 8, 2, 2]
    assert bench.seglen_of(4, full=False) == 8  # one-GPU rehearsal: a share of the CUs per rank
    monkeypatch.setenv("TQR_SEGLEN", "5")
    assert bench.seglen_of(8) == 5 and bench.seglen_of(1) == 5
