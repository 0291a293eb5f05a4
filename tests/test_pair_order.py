"""CPU check of the fp64 chain's paired reflector order (tiles.hpp sigp, flow.hpp image writer):
relabelling a group's reflectors by sigp keeps W = -T^T Z exact when the packed product skips
the k-blocks kb < (wi & ~1) — i.e. the permuted T is block-upper-triangular at 8-reflector
granularity — and the relabelling is a bijection onto the group's reflectors."""
import numpy as np
import pytest


def sigp(r, x):
    return 8 * (r >> 1) + 2 * x + (r & 1)


@pytest.mark.parametrize("ib", [16, 32])
def test_sigp_is_a_permutation(ib):
    nri = ib // 4
    got = sorted(sigp(r, x) for r in range(nri) for x in range(4))
    assert got == list(range(ib))
    # a lane's two head registers H[2h], H[2h+1] are consecutive rows (one 16-B access)
    for h in range(nri // 2):
        for x in range(4):
            assert sigp(2 * h + 1, x) == sigp(2 * h, x) + 1


@pytest.mark.parametrize("ib", [16, 32])
def test_packed_w_skips_only_zero_blocks(ib):
    nri = ib // 4
    rng = np.random.default_rng(7)
    T = np.triu(rng.standard_normal((ib, ib)))  # compact-WY T: upper triangular
    Z = rng.standard_normal((ib, 16))           # Z rows = reflectors, 16 strip columns
    # W[wi] block (rows sigp(wi, y), y < 4) = sum over k-blocks kb of (-T)[kb-block][wi-block]^T Z[kb-block]
    W = np.zeros((ib, 16))
    for wi in range(nri):
        rows = [sigp(wi, y) for y in range(4)]
        for kb in range(nri):
            if kb & ~1 > wi:  # the packed image's zero blocks (never multiplied)
                cols = [sigp(kb, x) for x in range(4)]
                assert not np.any(T[np.ix_(cols, rows)]), (wi, kb)
                continue
            cols = [sigp(kb, x) for x in range(4)]
            W[rows] += -T[np.ix_(cols, rows)].T @ Z[cols]
    np.testing.assert_allclose(W, -T.T @ Z, rtol=0, atol=1e-12)
