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
