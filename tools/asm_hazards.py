#!/usr/bin/env python3
"""gfx950 hazard audit of inline assembly in compiled device code (build step, with check_chain_asm.py).

The hand-scheduled chain statements (gen/gen_chain_asm.py, gen/gen_chain32_asm.py) bypass hipcc's
hazard recognizer: the generators pad the pairs of their own table, the compiler pads the pairs of
its own code, and nobody checks the pairs that straddle a `;;#ASMSTART` / `;;#ASMEND` boundary or
that the generators' table does not list. Round 5 lost a day to exactly that (a `v_readfirstlane` of
a VGPR written by the compiler's VALU move in the instruction before it).

This audit walks the control-flow graph of every function of the device assembly that contains
inline asm, tracks for every register the recent writes (which instruction class wrote it and how
many wait states ago, the minimum over all paths into a block), and checks every read against the
table in gen/gfx950_hazards.py (the generators' table). A pair is reported when at least one of its
two instructions comes from inline asm (pairs of compiled code are the compiler's; `--all` checks
those too, which tests the table against hipcc's own padding).

Usage: asm_hazards.py [--all] <device .s> [function-name-regex]
"""
import os
import re
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "gpu-tiled-qr-decomposition_amd", "gen"))
import gfx950_hazards as HZ  # noqa: E402

HORIZON = 20  # wait states after which no rule applies (the table's largest value is 18)

_REG = re.compile(r"^(v|s|a|ttmp)(?:\[(\d+):(\d+)\]|(\d+))$")
_DPP = ("row_", "quad_perm", "wave_", "bank_mask", "row_mask", "bound_ctrl")


def _regs(op):
    """Register keys named by one operand ('v12', 's[4:7]', 'vcc', 'exec', 'm0' ...)."""
    op = op.strip()
    if op in ("vcc", "vcc_lo", "vcc_hi"):
        return ["vcc"]
    if op in ("exec", "exec_lo", "exec_hi"):
        return ["exec"]
    if op == "m0":
        return ["m0"]
    m = _REG.match(op)
    if not m:
        return []
    kind = m.group(1)
    lo, hi = (int(m.group(4)),) * 2 if m.group(4) is not None else (int(m.group(2)), int(m.group(3)))
    return [f"{kind}{r}" for r in range(lo, hi + 1)]


def _split_operands(rest):
    """'v[1:2], v3, s[4:7], s5 offen offset:64 sc1' -> (['v[1:2]', 'v3', 's[4:7]', 's5'], 'offen ...')."""
    ops, depth, cur = [], 0, ""
    for ch in rest:
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == "," and depth == 0:
            ops.append(cur.strip())
            cur = ""
        else:
            cur += ch
    cur = cur.strip()
    mods = ""
    if cur:
        parts = cur.split(None, 1)
        ops.append(parts[0])
        mods = parts[1] if len(parts) > 1 else ""
    # a modifier may also follow an earlier operand's space (e.g. 'v97, off sc1')
    return [o.split()[0] if o else o for o in ops], mods


class Insn:
    """One instruction: its class, wait states, and the registers it reads (by role) and writes."""

    def __init__(self, text, line, in_asm):
        self.text, self.line, self.in_asm = text, line, in_asm
        parts = text.split(None, 1)
        self.op = parts[0]
        self.ops, self.mods = _split_operands(parts[1]) if len(parts) > 1 else ([], "")
        self.waits = 1
        self.reads = []    # (reg, role)
        self.writes = []   # reg
        self.cls = "other"
        self.target = None  # branch target label
        self.cond = False   # conditional branch (falls through)
        self.term = False   # ends the block without fall-through
        self._classify()

    def _r(self, i, role):
        if i < len(self.ops):
            self.reads += [(r, role) for r in _regs(self.ops[i])]

    def _w(self, i):
        if i < len(self.ops):
            self.writes += _regs(self.ops[i])

    def _classify(self):
        op, n = self.op, len(self.ops)
        if op == "s_nop":
            self.cls, self.waits = "nop", int(self.ops[0], 0) + 1
        elif op in ("s_branch", "s_setpc_b64") or op.startswith("s_cbranch"):
            self.cls = "branch"
            if op == "s_setpc_b64":
                self.term = True  # (a return, or a long branch: its target is resolved by the caller)
                self._r(0, "salu")
            else:
                self.target = self.ops[0] if self.ops else None
                self.cond = op != "s_branch"
                self.term = not self.cond
        elif op == "s_endpgm":
            self.cls, self.term = "branch", True
        elif op.startswith(("v_mfma", "v_smfmac")):
            self.cls = "mfma"
            self._w(0)
            self._r(1, "srcab")
            self._r(2, "srcab")
            self._r(3, "srcc")
        elif op in ("v_readfirstlane_b32", "v_readlane_b32"):
            self.cls = "readlane"
            self._w(0)
            self._r(1, "readlane")
            self._r(2, "lanesel")
        elif op == "v_writelane_b32":
            self.cls = "readlane"
            self._w(0)
            self._r(1, "valu")
            self._r(2, "lanesel")
        elif op.startswith("v_"):
            self.cls = "valu"
            self._w(0)
            first = 1
            if any(t in op for t in ("_co_", "mad_u64_u32", "mad_i64_i32", "div_scale")) and n > 1 and \
                    (self.ops[1].startswith("s") or self.ops[1].startswith("vcc")):
                self._w(1)
                first = 2
            dpp = any(self.mods.startswith(p) or (" " + p) in self.mods for p in _DPP)
            for i in range(first, n):
                self._r(i, "dpp" if dpp and i == first else "valu")
            if op.startswith("v_cmpx"):
                self.writes.append("exec")
        elif op.startswith(("buffer_", "global_", "flat_", "scratch_")):
            self._vmem()
        elif op.startswith("ds_"):
            self.cls = "ds"
            if op.startswith(("ds_read", "ds_load", "ds_bpermute", "ds_permute", "ds_swizzle", "ds_append", "ds_consume")):
                self._w(0)
                for i in range(1, n):
                    self._r(i, "vmem_addr")
            else:
                for i in range(n):
                    self._r(i, "vmem_addr")
        elif op.startswith("s_set_gpr_idx_on"):
            self.cls = "gpr_idx_on"
            self._r(0, "salu")
            self.writes.append("m0")
        elif op.startswith(("s_load", "s_buffer_load", "s_memrealtime", "s_memtime", "s_getpc")):
            self.cls = "smem"
            self._w(0)
        elif op.startswith("s_"):
            self.cls = "salu"
            if op.startswith(("s_cmp", "s_bitcmp", "s_waitcnt", "s_barrier", "s_setprio", "s_sleep", "s_sendmsg",
                              "s_set_gpr_idx_off", "s_icache", "s_trap", "s_ttrace")):
                for i in range(n):
                    self._r(i, "salu")
            else:
                self._w(0)
                for i in range(1, n):
                    self._r(i, "salu")
                if "saveexec" in op:
                    self.writes.append("exec")

    def _vmem(self):
        op, n = self.op, len(self.ops)
        lds = "_lds_" in op or re.search(r"(^|\s)lds(\s|$)", self.mods) is not None
        store = "_store" in op
        atomic = "_atomic" in op
        self.cls = "lds_dma" if lds else "store" if store or atomic else "load"
        if op.startswith("buffer_"):
            if lds:
                roles = ["vmem_addr"] * n  # (vdata slot unused: 'off' or a dummy)
            elif store or (atomic and not re.search(r"\b(sc0|glc)\b", self.mods)):
                roles = ["store_data"] + ["vmem_addr"] * (n - 1)
            else:
                roles = ["w"] + ["vmem_addr"] * (n - 1)
        elif op.startswith("global_load_lds") or op.startswith("scratch_load_lds"):
            roles = ["vmem_addr"] * n
        elif op.startswith(("global_store", "flat_store", "scratch_store")):
            roles = ["vmem_addr", "store_data"] + ["vmem_addr"] * (n - 2)
        elif atomic:
            ret = re.search(r"\b(sc0|glc)\b", self.mods) is not None
            roles = (["w", "vmem_addr", "store_data"] if ret else ["vmem_addr", "store_data"]) + ["vmem_addr"] * n
        else:  # loads
            roles = ["w"] + ["vmem_addr"] * (n - 1)
        for i in range(n):
            if roles[i] == "w":
                self._w(i)
            else:
                self._r(i, roles[i])
        if lds:
            self.reads.append(("m0", "lds_dma"))


def _required(w_cls, w_op, reg, insn, role, hw=False, w_d=None):
    """Wait states the write (class w_cls, opcode w_op) of reg needs before insn reads it as role
    (hw: the hardware's own requirement where the generators keep a margin above it)."""
    vec = reg[0] in "va"
    if w_cls == "mfma":
        t = (HZ.MFMA_HW if hw else HZ.MFMA).get(w_op, HZ.MFMA_DEFAULT)
        if insn.cls == "mfma":
            if role == "srcc" and hw and insn.op == w_op and insn.ops[3] == w_d:
                return t["srcc_same"]  # (an accumulation chain: srcC is exactly the writer's D)
            return t["srcc"] if role == "srcc" else t["srcab"]
        if insn.cls in ("valu", "readlane"):
            return t["valu"]
        if role == "store_data" or insn.cls in ("ds", "load", "store", "lds_dma"):
            return t["vmem"]  # (as VMEM / LDS data or address: ds_bpermute of the strip, ds_write of a result)
        return 0
    if w_cls in ("valu", "readlane"):
        if vec:
            if insn.cls == "mfma":
                return HZ.VALU_TO_MFMA
            if role == "store_data":
                return 0 if hw else HZ.VALU_TO_STORE
            if role == "readlane":
                return HZ.VALU_VGPR_TO_READLANE
            if role == "dpp":
                return HZ.VALU_VGPR_TO_DPP
            return 0
        # an SGPR / VCC written by a VALU (v_readfirstlane, v_cmp, a carry-out)
        if insn.cls in ("load", "store", "lds_dma"):
            return HZ.VALU_SGPR_TO_VMEM
        if role == "lanesel":
            return HZ.VALU_SGPR_TO_LANESEL
        if insn.cls in ("valu", "readlane", "mfma"):
            return HZ.VALU_SGPR_TO_VALU
        return 0
    if w_cls == "salu" and reg == "m0" and role == "lds_dma":
        return HZ.M0_TO_LDS_DMA
    if w_cls == "gpr_idx_on" and insn.cls in ("valu", "mfma") and reg == "__gpr_idx":
        return HZ.GPR_IDX_ON_TO_VALU
    return 0


def parse_functions(text):
    """{function name: [(line number, text), ...]} for every function of the .s."""
    lines = text.split("\n")
    funcs, cur, name = {}, None, None
    for i, l in enumerate(lines):
        m = re.match(r"^([A-Za-z_.$][\w.$]*):", l)
        if m and not l.startswith(".L") and not l.startswith(" ") and not l.startswith("\t"):
            name = m.group(1)
            if not name.startswith("."):
                cur = funcs.setdefault(name, [])
                continue
        if l.startswith(".Lfunc_end"):
            cur = None
            continue
        if cur is not None:
            cur.append((i + 1, l))
    return funcs


def build_insns(body):
    """Instructions and labels of one function, in layout order: [('label', name) | ('insn', Insn)]."""
    out, in_asm, asm_id = [], False, 0
    for ln, l in body:
        s = l.strip()
        if ";;#ASMSTART" in s:
            in_asm, asm_id = True, asm_id + 1
            out.append(("asmstart", asm_id))
            continue
        if ";;#ASMEND" in s:
            in_asm = False
            out.append(("asmend", asm_id))
            continue
        code = s.split(";")[0].strip()
        if not code or code.startswith("."):
            if re.match(r"^\.L[\w$.]*:", code):
                out.append(("label", code[:-1]))
            continue
        # several statements on one line ('1: s_nop 0') and local labels
        while True:
            m = re.match(r"^([0-9]+|[A-Za-z_.$][\w.$]*):\s*(.*)$", code)
            if not m:
                break
            lab = m.group(1)
            out.append(("label", (asm_id, lab) if lab.isdigit() else lab))
            code = m.group(2)
        if code:
            out.append(("insn", Insn(code, ln, in_asm)))
    return out


def _resolve_targets(items):
    """Branch targets -> index of the label item; local numeric labels ('1f' / '1b') resolve inside their asm block."""
    label_at = {}
    for idx, (k, v) in enumerate(items):
        if k == "label" and not isinstance(v, tuple):
            label_at[v] = idx
    locals_ = [(idx, v) for idx, (k, v) in enumerate(items) if k == "label" and isinstance(v, tuple)]
    tgt = {}
    for idx, (k, v) in enumerate(items):
        if k != "insn" or v.cls != "branch":
            continue
        t = v.target
        if t is None:
            # s_setpc_b64 of a long branch: its target is named by the s_add_u32 before it
            for j in range(idx - 1, max(idx - 4, -1), -1):
                kk, vv = items[j]
                if kk == "insn":
                    m = re.search(r"\((\.L\w+)-", vv.text)
                    if m:
                        tgt[idx] = label_at.get(m.group(1))
                        break
            continue
        m = re.match(r"^(\d+)([fb])$", t)
        if m:
            n, d = m.group(1), m.group(2)
            cands = [i for i, (aid, lab) in locals_ if lab == n]
            if d == "f":
                nxt = [i for i in cands if i > idx]
                tgt[idx] = nxt[0] if nxt else None
            else:
                prv = [i for i in cands if i < idx]
                tgt[idx] = prv[-1] if prv else None
        else:
            tgt[idx] = label_at.get(t)
    return tgt


def _merge(a, b):
    """State merge: per (register, writer) the fewest wait states since the write."""
    out = dict(a)
    for key, rec in b.items():
        if key not in out or rec[0] < out[key][0]:
            out[key] = rec
    return out


def _advance(state, n):
    out = {}
    for key, (d, line, in_asm, dt) in state.items():
        d2 = d + n
        if d2 <= HORIZON:
            out[key] = (d2, line, in_asm, dt)
    return out


def _mubuf_soffset_reg(insn):
    """A buffer_* store whose soffset operand (the 4th: vdata, vaddr, srsrc, soffset) is an SGPR."""
    return insn.op.startswith("buffer_") and len(insn.ops) > 3 and re.match(r"s\d+$|s\[", insn.ops[3]) is not None


def _store_bytes(op):
    m = re.search(r"_(?:dword|b)(x?\d*)$", op.split("_lds")[0])
    if op.endswith(("_dwordx4", "_b128")):
        return 16
    if op.endswith(("_dwordx3", "_b96")):
        return 12
    if op.endswith(("_dwordx2", "_b64")):
        return 8
    return 4 if m else 4


STATS = {"pairs": 0}


def _step(state, insn, report, hw=False):
    """Check insn's reads against state, then apply its writes. state: {(reg, w_cls, w_op): (dist, line, in_asm)}."""
    reads = list(insn.reads)
    if insn.cls in ("valu", "mfma"):
        reads.append(("__gpr_idx", "valu"))
    by_reg = {}
    for key, rec in state.items():
        by_reg.setdefault(key[0], []).append((key, rec))
    for reg, role in reads:
        for (r, w_cls, w_op), (dist, wline, w_asm, w_d) in by_reg.get(reg, []):
            if w_cls == "store_read":
                continue
            req = _required(w_cls, w_op, reg, insn, role, hw, w_d)
            if report.__name__ == "report_rec":
                STATS["pairs"] += 1
            if req > dist:
                report(insn, wline, w_asm, f"{w_cls} {w_op} -> {insn.op} ({role} {reg}): {dist} of {req} wait states")
    # write-after-read of a store's data VGPRs
    for reg in insn.writes:
        for (r, w_cls, w_op), (dist, wline, w_asm, w_soff) in by_reg.get(reg, []):
            # (hardware: a MUBUF store whose soffset is a register has no data hazard — the rule
            # of LLVM's GCNHazardRecognizer::createsVALUHazard, which hipcc pads by)
            need = (HZ.STORE_WAR_HW if _store_bytes(w_op) > 8 and insn.cls != "load" and not w_soff else 0) \
                if hw else HZ.STORE_WAR
            if w_cls == "store_read" and insn.cls in ("valu", "mfma", "readlane", "load") and need > dist:
                report(insn, wline, w_asm, f"store data {reg} of {w_op} overwritten by {insn.op}: {dist} of {need} wait states")
    state = _advance(state, insn.waits)
    if insn.cls not in ("nop", "branch"):
        for reg in insn.writes:
            for key in [k for k in state if k[0] == reg]:
                del state[key]
            state[(reg, insn.cls, insn.op)] = (0, insn.line, insn.in_asm, insn.ops[0] if insn.ops else None)
        if insn.cls == "gpr_idx_on":
            state[("__gpr_idx", "gpr_idx_on", insn.op)] = (0, insn.line, insn.in_asm, None)
        for reg, role in insn.reads:
            if role == "store_data":
                state[(reg, "store_read", insn.op)] = (0, insn.line, insn.in_asm, _mubuf_soffset_reg(insn))
    return state


def check_function(items, all_pairs=False):
    """Violations [(reader line, writer line, message)] of one function's instruction list."""
    tgt = _resolve_targets(items)
    n = len(items)
    # basic blocks: leaders at labels and after branches
    leaders = {0}
    for idx, (k, v) in enumerate(items):
        if k == "label":
            leaders.add(idx)
        if k == "insn" and v.cls == "branch":
            leaders.add(idx + 1)
    starts = sorted(x for x in leaders if x < n)
    block_of = {}
    blocks = []
    for bi, s0 in enumerate(starts):
        e0 = starts[bi + 1] if bi + 1 < len(starts) else n
        blocks.append((s0, e0))
        for x in range(s0, e0):
            block_of[x] = bi
    succ = [[] for _ in blocks]
    for bi, (s0, e0) in enumerate(blocks):
        last = items[e0 - 1] if e0 > s0 else None
        falls = True
        if last and last[0] == "insn" and last[1].cls == "branch":
            t = tgt.get(e0 - 1)
            if t is not None:
                succ[bi].append(block_of[t])
            falls = not last[1].term
        if falls and bi + 1 < len(blocks):
            succ[bi].append(bi + 1)
    entry = [None] * len(blocks)
    entry[0] = {}
    violations = {}

    def run_block(bi, record):
        st = dict(entry[bi])
        s0, e0 = blocks[bi]
        for x in range(s0, e0):
            k, v = items[x]
            if k != "insn":
                continue

            def report_rec(insn, wline, w_asm, msg):
                if all_pairs or insn.in_asm or w_asm:
                    violations[(insn.line, wline, msg)] = None

            def report(insn, wline, w_asm, msg):
                pass
            st = _step(st, v, report_rec if record else report, all_pairs)
        return st

    work = [0]
    while work:
        bi = work.pop()
        out = run_block(bi, False)
        for sb in succ[bi]:
            new = out if entry[sb] is None else _merge(entry[sb], out)
            if entry[sb] is None or new != entry[sb]:
                entry[sb] = new
                work.append(sb)
    for bi in range(len(blocks)):
        if entry[bi] is not None:
            run_block(bi, True)
    return sorted(violations)


def check_text(text, name_re=None, all_pairs=False):
    """{function: violations} over the functions of an assembly text that contain inline asm."""
    res = {}
    for name, body in parse_functions(text).items():
        if name_re and not re.search(name_re, name):
            continue
        if not any(";;#ASMSTART" in l for _, l in body):
            continue
        res[name] = check_function(build_insns(body), all_pairs)
    return res


def main(argv):
    all_pairs = "--all" in argv
    args = [a for a in argv if a != "--all"]
    text = open(args[0]).read()
    res = check_text(text, args[1] if len(args) > 1 else None, all_pairs)
    bad = 0
    quiet = len(res) > 8  # (the build: one summary line, the offending functions in full)
    for name, v in res.items():
        if v or not quiet:
            print(f"asm_hazards: {name[:90]}: {'ok' if not v else f'{len(v)} violations'}")
        for rl, wl, msg in v[:20]:
            print(f"    line {rl} (after line {wl}): {msg}")
        bad += len(v)
    print(f"asm_hazards: {len(res)} functions with inline asm, {STATS['pairs']} register pairs within the hazard "
          f"window checked, {bad} violations")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
