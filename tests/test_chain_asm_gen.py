"""The hand-scheduled fp64 chain's generator (gpu-tiled-qr-decomposition_amd/gen/gen_chain_asm.py).

CPU-only: regenerating the statement text must reproduce the committed chain_asm_gen.inc (the build
compiles the committed file), and the generator's own simulation of the counted waits
(`simulate`: every LDS-DMA, strip, head-row and store operation complete at the wait that needs it,
for chains of 1, 2, 3 and 5 elements, tiles of 128 and 256) runs inside `main` and must pass."""
import importlib.util
import pathlib

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
PKG = ROOT / "gpu-tiled-qr-decomposition_amd"


def _gen():
    spec = importlib.util.spec_from_file_location("gen_chain_asm", PKG / "gen" / "gen_chain_asm.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_generated_text_is_committed(tmp_path, monkeypatch):
    g = _gen()
    out = tmp_path / "chain_asm_gen.inc"
    monkeypatch.setattr("sys.argv", ["gen_chain_asm.py", str(out)])
    g.main()
    assert out.read_text() == (PKG / "csrc" / "chain_asm_gen.inc").read_text()


@pytest.mark.parametrize("B", [128, 256])
def test_wait_counts_simulated(B):
    g = _gen()
    bodies = []
    for ho in (False, True):
        b = g.Body(B, ho)
        b.build()
        bodies.append(b)
    for n in (1, 2, 4):
        assert g.simulate(B, tuple(bodies), nelem=n)


@pytest.mark.parametrize("B", [128, 256])
def test_statement_registers(B):
    """Every register a statement names is one the statements own (v32..v255) or an operand."""
    import re
    g = _gen()
    for ho in (False, True):
        b = g.Body(B, ho)
        s = b.build()
        for line in s.lines:
            for m in re.finditer(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b", line):
                lo = int(m.group(1) or m.group(3))
                assert lo >= g.VLO, line
            assert "a[" not in line and not re.search(r"\bs\d+\b", line), line


def _ubodies(g, B, late):
    NG, lead = B // g.IB, g.XLEAD
    ub = {}
    for gg in range(1, NG):
        if gg + 1 < NG:
            ub[gg] = g.Body(B, False, skip=8 * gg, early_st=range(4 * (gg - 1), 4 * gg))
        else:
            ub[gg] = g.Body(B, True, xlead=lead if late else None, skip=8 * gg, early_st=range(4 * (gg - 1), 4 * gg),
                            early_ld=[p for p in range(4 * gg) if not late or p < lead])
        ub[gg].build()
    return ub


@pytest.mark.parametrize("B", [128, 256])
@pytest.mark.parametrize("late", [False, True])
def test_unmqr_bodies(B, late):
    """UNMQR element (GE-type V, zero above group g's rows): group g runs k-steps >= 8 g only —
    (NKS - 8 g) x 8 MFMAs in each phase plus the T-multiplication's 40 — stores the rows group g-1
    finished, and the chain's waits still cover every operation (strip stored / next strip loaded
    exactly once per row pair, checked by simulate) with the hand-over's own sync count."""
    import re
    g = _gen()
    NKS = B // 4
    ub = _ubodies(g, B, late)
    for gg, b in ub.items():
        nm = sum(1 for l in b.s.lines if l.startswith("v_mfma"))
        assert nm == 2 * 8 * (NKS - 8 * gg) + 40
        for line in b.s.lines:
            for m in re.finditer(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b", line):
                assert int(m.group(1) or m.group(3)) >= g.VLO, line
    plain, ho = g.Body(B, False), g.Body(B, True, xlead=g.XLEAD if late else None)
    plain.build()
    ho.build()
    bodies = (plain, ho)
    if late:
        xb = g.Body(B, False, xin_from=g.XLEAD)
        xb.build()
        bodies = (plain, ho, xb)
    for n in (1, 2, 4):
        assert g.simulate(B, bodies, nelem=n, ubodies=ub)
    # the plain hand-over's sync count would leave the UNMQR hand-over's LDS-DMA in flight: the
    # engine uses the generated TQR_CHAIN_ASM_UHANDOVER*_SYNC_B* after an UNMQR element
    assert ub[B // g.IB - 1].sync_after() < ho.sync_after()


def _gen32():
    spec = importlib.util.spec_from_file_location("gen_chain32_asm", PKG / "gen" / "gen_chain32_asm.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_chain32_generated_text_is_committed(tmp_path, monkeypatch):
    """fp32 chain statements (gen_chain32_asm.py): the committed chain32_asm_gen.inc is current."""
    g = _gen32()
    out = tmp_path / "chain32_asm_gen.inc"
    monkeypatch.setattr("sys.argv", ["gen_chain32_asm.py", str(out)])
    g.main()
    assert out.read_text() == (PKG / "csrc" / "chain32_asm_gen.inc").read_text()


@pytest.mark.parametrize("B", [128, 256])
def test_chain32_bodies(B):
    """fp32 bodies: MFMA counts (phase 1 and 2: 8 per tile, T: 12; UNMQR group g skips 2 g tiles),
    registers within the statements' range, and the counted waits of chains of 1-5 elements with
    both hand-over forms (simulate: each group's LDS-DMA at its sync point, each strip tile before
    its first MFMA, every strip stored and loaded exactly once)."""
    import re
    g = _gen32()
    NMT = B // 16
    plain, ho, hol, xb = g.Body32(B), g.Body32(B, handover=True), g.Body32(B, handover=True, xlead=g.XLEAD), g.Body32(B, xin_from=g.XLEAD)
    bodies = [plain, ho, hol, xb] + [g.Body32(B, ts=False, k0=2 * u) for u in range(B // 32)]
    for b in bodies:
        b.build()
        nm = sum(1 for l in b.s.lines if l.startswith("v_mfma"))
        assert nm == 2 * 8 * (NMT - b.k0) + 12
        for line in b.s.lines:
            for m in re.finditer(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b", line):
                assert int(m.group(1) or m.group(3)) >= g.VLO, line
    for n in (1, 2, 3, 5):
        assert g.simulate(B, plain, ho, None, n)
        assert g.simulate(B, plain, hol, xb, n)
