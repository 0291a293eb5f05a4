#!/usr/bin/env python3
"""Audit of the fp64 asm chain in the compiled device assembly (build step, see Makefile).

The hand-scheduled chain statements (csrc/chain_asm.hpp, gen/gen_chain_asm.py) keep the strip and
the head rows in v[32:255] BETWEEN statements, where the compiler does not know they are live (each
statement merely clobbers them). That is only correct if no compiled instruction of flow_chain_asm
that runs while a strip is live touches those registers. This script checks a stronger property,
independent of the control flow, on the assembly hipcc produced (-save-temps), for every
instantiation of flow_chain_asm:
  * no instruction outside an inline-asm block reads or writes a VGPR >= v32 (or an AGPR);
  * no scratch access between the first and the last inline-asm block (a spill reload would wait
    for the wave's whole memory queue), and no call anywhere.
and, since round 6, the gfx950 hazard audit of every function with inline asm (tools/asm_hazards.py:
every instruction pair in which one side is inline asm — inside the chain statements and across their
boundaries with compiled code — against the wait-state table the generators pad with,
gen/gfx950_hazards.py).
Exit status 1 with the offending lines otherwise.
Usage: check_chain_asm.py <device .s>
"""
import os
import re
import sys

VLO = 32  # first register owned by the chain statements (gen_chain_asm.py VLO)
REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+))\b")


def regs(line):
    out = []
    for m in REG.finditer(line):
        kind = m.group(1)
        if m.group(4) is not None:
            lo = hi = int(m.group(4))
        else:
            lo, hi = int(m.group(2)), int(m.group(3))
        out.append((kind, lo, hi))
    return out


def check(path):
    lines = open(path).read().split("\n")
    starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\S*flow_chain(?:32)?_(asm|res)\S*:", l)]
    if not starts:
        print("check_chain_asm: no flow_chain_asm in", path)
        return 1
    bad = 0
    for st in starts:
        name = lines[st].split(":")[0]
        end = next((i for i in range(st + 1, len(lines)) if lines[i].startswith(".Lfunc_end")), len(lines))
        last = max((i for i in range(st, end) if ";;#ASMSTART" in lines[i]), default=end)
        inasm, armed, errs = False, False, []
        for i in range(st + 1, end):
            l = lines[i]
            if ";;#ASMSTART" in l:
                inasm = True
                continue
            if ";;#ASMEND" in l:
                inasm = False
                continue
            code = l.split(";")[0].strip()
            if not code or code.startswith(".") or code.endswith(":"):
                continue
            rs = regs(code)
            if inasm:
                armed = True
                continue
            if any(k == "a" or (k == "v" and hi >= VLO) for k, lo, hi in rs):
                errs.append(f"{i + 1}: {code}")
            elif "s_swappc" in code or (armed and code.startswith("scratch_") and i < last):
                errs.append(f"{i + 1}: {code}")
        status = "ok" if not errs else f"{len(errs)} violations"
        print(f"check_chain_asm: {name[:90]}: {status}")
        for e in errs[:30]:
            print("   ", e)
        bad += len(errs)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import asm_hazards
    rc_regs = check(sys.argv[1])
    rc_hz = asm_hazards.main([sys.argv[1]])
    sys.exit(1 if rc_regs or rc_hz else 0)
