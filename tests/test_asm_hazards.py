"""The build's gfx950 hazard audit of inline asm (tools/asm_hazards.py, run by check_chain_asm.py in the
Makefile on the compiled device assembly), CPU-only.

* seeded violations: one snippet per hazard class the generated chain statements rely on (the
  round-5 one first: a VALU write of a VGPR, then `v_readfirstlane` of it at a statement's start)
  must be reported, and the same snippet with the table's wait states must pass;
* every generated statement (chain_asm_gen.inc, chain32_asm_gen.inc), its operands bound to
  registers, passes alone and back to back with itself around a loop (the pairs across two
  statements), and the audit finds nothing in them with a margin shaved off (it really reads them);
* the compiled assembly, when a build left it in-tree, passes (the same check the build runs)."""
import importlib.util
import pathlib
import re

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
PKG = ROOT / "gpu-tiled-qr-decomposition_amd"


def _mod(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


AH = _mod("asm_hazards", ROOT / "tools" / "asm_hazards.py")
HZ = AH.HZ


def _func(body_lines, asm=None):
    """A one-function assembly text; lines between '<asm>' and '</asm>' markers are inline asm."""
    out = ["fn:"]
    for l in body_lines:
        if l == "<asm>":
            out.append("\t;;#ASMSTART")
        elif l == "</asm>":
            out.append("\t;;#ASMEND")
        else:
            out.append("\t" + l)
    out += ["\ts_setpc_b64 s[30:31]", ".Lfunc_end0:"]
    return "\n".join(out)


def _violations(lines):
    res = AH.check_text(_func(lines))
    return res.get("fn", [])


def _nops(n):
    return [f"s_nop {n - 1}"] if n > 0 else []


# (name, writer lines, reader lines, required wait states)
CASES = [
    ("valu vgpr -> readfirstlane (round 5)", ["v_mov_b32_e32 v5, s3"], ["<asm>", "v_readfirstlane_b32 s4, v5", "</asm>"],
     HZ.VALU_VGPR_TO_READLANE),
    ("valu sgpr -> vmem", ["<asm>", "v_readfirstlane_b32 s7, v1", "</asm>"],
     ["<asm>", "buffer_load_dwordx4 v[40:43], v2, s[8:11], s7 offen", "</asm>"], HZ.VALU_SGPR_TO_VMEM),
    ("valu sgpr -> valu", ["v_readfirstlane_b32 s7, v1"], ["<asm>", "v_add_u32 v40, s7, v2", "</asm>"], HZ.VALU_SGPR_TO_VALU),
    ("valu sgpr -> lane select", ["v_readfirstlane_b32 s7, v1"], ["<asm>", "v_readlane_b32 s8, v40, s7", "</asm>"],
     HZ.VALU_SGPR_TO_LANESEL),
    ("m0 -> lds-dma", ["s_mov_b32 m0, s5"], ["<asm>", "global_load_lds_dwordx4 v97, s[2:3] sc1", "</asm>"], HZ.M0_TO_LDS_DMA),
    ("gpr_idx_on -> valu", ["<asm>", "s_set_gpr_idx_on s6, gpr_idx(SRC0)"], ["v_add_f64 v[80:81], v[128:129], v[80:81]",
                                                                            "s_set_gpr_idx_off", "</asm>"],
     HZ.GPR_IDX_ON_TO_VALU),
    ("mfma f64 -> valu", ["<asm>", "v_mfma_f64_4x4x4_4b_f64 v[80:81], v[32:33], v[128:129], 0"],
     ["v_add_f64 v[112:113], v[112:113], v[80:81]", "</asm>"], HZ.F64["valu"]),
    ("mfma f64 -> store data", ["<asm>", "v_mfma_f64_4x4x4_4b_f64 v[128:129], v[32:33], v[96:97], v[128:129]"],
     ["buffer_store_dwordx4 v[128:131], v6, s[8:11], 0 offen", "</asm>"], HZ.F64["vmem"]),
    ("mfma f64 -> srcA", ["<asm>", "v_mfma_f64_4x4x4_4b_f64 v[80:81], v[32:33], v[128:129], 0"],
     ["v_mfma_f64_4x4x4_4b_f64 v[96:97], v[80:81], v[34:35], 0", "</asm>"], HZ.F64["srcab"]),
    ("mfma f32 -> srcB", ["<asm>", "v_mfma_f32_16x16x4_f32 v[80:83], v32, v128, 0"],
     ["v_mfma_f32_16x16x4_f32 v[96:99], v33, v80, 0", "</asm>"], HZ.F32["srcab"]),
    ("valu -> mfma", ["v_mov_b32_e32 v40, 0"], ["<asm>", "v_mfma_f64_4x4x4_4b_f64 v[80:81], v[40:41], v[128:129], 0", "</asm>"],
     HZ.VALU_TO_MFMA),
    ("store data -> overwrite", ["<asm>", "buffer_store_dwordx4 v[112:115], v6, s[8:11], 0 offen"],
     ["v_mov_b32_e32 v112, 0", "</asm>"], HZ.STORE_WAR),
]


@pytest.mark.parametrize("name,wr,rd,req", CASES, ids=[c[0] for c in CASES])
def test_seeded_violation_is_reported(name, wr, rd, req):
    assert req >= 1
    v = _violations(wr + rd)
    assert v, f"{name}: back to back and not reported"
    if req > 1:
        assert _violations(wr + _nops(req - 1) + rd), f"{name}: {req - 1} wait states and not reported"
    assert not _violations(wr + _nops(req) + rd), f"{name}: {req} wait states and still reported"


def test_compiled_pairs_are_the_compilers():
    """A pair of two compiled instructions is not the audit's (hipcc pads its own), unless --all."""
    lines = ["v_mov_b32_e32 v5, s3", "v_readfirstlane_b32 s4, v5", "<asm>", "s_nop 0", "</asm>"]
    assert not _violations(lines)
    assert AH.check_text(_func(lines), all_pairs=True)["fn"]


def test_store_war_soffset_register_exception():
    """Hardware rule (--all): a >8-byte MUBUF store whose soffset is an SGPR has no data hazard (hipcc
    pads none); with a constant soffset, or a global store, one wait state is needed."""
    rd = ["v_cndmask_b32_e64 v0, v15, v14, s[72:73]"]
    sgpr = ["<asm>", "buffer_store_dwordx4 v[0:3], v36, s[48:51], s68 offen sc1", "</asm>"]
    const = ["<asm>", "buffer_store_dwordx4 v[0:3], v36, s[48:51], 0 offen sc1", "</asm>"]
    glob = ["<asm>", "global_store_dwordx4 v[40:41], v[0:3], off sc1", "</asm>"]
    assert not AH.check_text(_func(sgpr + rd), all_pairs=True)["fn"]
    assert AH.check_text(_func(const + rd), all_pairs=True)["fn"]
    assert AH.check_text(_func(glob + rd), all_pairs=True)["fn"]
    # the generators' own margin (default mode) applies to every store
    assert _violations(sgpr[:-1] + rd + ["</asm>"])


def test_hazard_across_a_back_edge():
    """The pair is only formed around the loop: the statement's last MFMA, the next iteration's first read."""
    lines = [".LBB0_1:", "<asm>", "v_add_f64 v[112:113], v[112:113], v[80:81]", "s_nop 7",
             "v_mfma_f64_4x4x4_4b_f64 v[80:81], v[32:33], v[128:129], 0", "</asm>", "s_cbranch_scc1 .LBB0_1"]
    v = _violations(lines)
    assert v and "v_add_f64" in v[0][2]
    fixed = lines[:-1] + ["s_nop 4"] + lines[-1:]
    assert not _violations(fixed)


def test_local_labels_inside_a_statement():
    """'1f' / '2f' branches inside a statement: both paths into the join are checked."""
    lines = ["<asm>", "s_cmp_eq_u32 s5, 0", "s_cbranch_scc1 1f",
             "v_mfma_f64_4x4x4_4b_f64 v[80:81], v[32:33], v[128:129], 0", "s_branch 2f", "1:", "s_nop 9", "2:",
             "v_add_f64 v[112:113], v[112:113], v[80:81]", "</asm>"]
    assert _violations(lines)
    ok = lines[:4] + ["s_nop 5"] + lines[4:]
    assert not _violations(ok)


def _statements(inc):
    """{macro name: statement text} of a generated .inc (C string-literal macros)."""
    text = (PKG / "csrc" / inc).read_text()
    out = {}
    for m in re.finditer(r'#define (TQR_\w+) ((?:"(?:[^"\\]|\\.)*"\s*\\?\s*)+)', text):
        parts = re.findall(r'"((?:[^"\\]|\\.)*)"', m.group(2))
        s = "".join(parts).replace("\\n", "\n").replace("\\t", "\t")
        if "\n" in s or "v_mfma" in s:
            out[m.group(1)] = s
    return out


# operands of the statements (chain_asm.hpp / chain32_asm.hpp / chain_res.hpp), bound to registers the
# compiler could use for them
BIND = {"vz": "v1", "vx": "v2", "vt": "v3", "vl16": "v4", "loff": "v5", "svsrc": "s[2:3]", "stsrc": "s[4:5]",
        "sdst": "s6", "sw": "s7", "hrs": "s[8:11]", "goff": "s12", "hsc": "s13", "xout": "s[16:19]",
        "xin": "s[20:23]", "hnx": "s[24:27]", "m0s": "s28", "st": "s29", "gidx": "s30", "rso": "s[32:35]",
        "rsi": "s[36:39]", "xs": "s40", "xso": "s41", "hso": "s42", "va0": "v6", "va1": "v7",
        "vb0": "v8", "vb1": "v9", "hnul": "s[60:63]"}


def _bind(stmt):
    def sub(m):
        return BIND[m.group(1)]
    return re.sub(r"%\[(\w+)\]", sub, stmt)


@pytest.mark.parametrize("inc", ["chain_asm_gen.inc", "chain32_asm_gen.inc"])
def test_generated_statements_pass(inc):
    stmts = _statements(inc)
    assert len(stmts) >= 10
    for name, s in stmts.items():
        body = [l.strip() for l in _bind(s).split("\n") if l.strip()]
        alone = ["<asm>"] + body + ["</asm>"]
        assert not _violations(alone), (name, _violations(alone)[:3])
        # back to back around a loop: the pairs between one statement's end and the next one's start
        looped = [".LBB0_9:"] + alone + ["s_cbranch_scc1 .LBB0_9"]
        assert not _violations(looped), (name, _violations(looped)[:3])


def test_generated_statements_are_read():
    """Shaving one wait state off the generator's padding is caught where the padding is tight: the
    audit parses the statements' registers, it does not pass them vacuously."""
    stmts = _statements("chain_asm_gen.inc")
    body = [l.strip() for l in _bind(stmts["TQR_CHAIN_ASM_PLAIN_B256"]).split("\n") if l.strip()]
    hits = 0
    for i, l in enumerate(body):
        m = re.match(r"s_nop (\d+)$", l)
        if m:
            shaved = body[:i] + ([f"s_nop {int(m.group(1)) - 1}"] if int(m.group(1)) > 0 else []) + body[i + 1:]
            if _violations(["<asm>"] + shaved + ["</asm>"]):
                hits += 1
    assert hits >= 3, hits


def test_compiled_assembly_passes():
    s = PKG / "build" / "engine-hip-amdgcn-amd-amdhsa-gfx950.s"
    if not s.exists():
        pytest.skip("no in-tree build (the Makefile runs the same check on every build)")
    res = AH.check_text(s.read_text())
    assert len(res) > 10
    assert not any(res.values()), {k: v[:3] for k, v in res.items() if v}
