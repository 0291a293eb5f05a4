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
