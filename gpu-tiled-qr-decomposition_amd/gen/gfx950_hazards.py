"""gfx950 (CDNA4) wait states of the instruction pairs the hand-scheduled chain statements rely on.

One table, used by the two generators (gen_chain_asm.py, gen_chain32_asm.py: they pad their own
statements with it) and by the build's hazard audit (tools/check_chain_asm.py: it checks every pair
of the compiled device assembly in which at least one side is inline asm — inside a statement and
across every ;;#ASMSTART / ;;#ASMEND boundary — against it). Wait states are counted as the
hardware does: one per issued instruction, n + 1 for `s_nop n`.

Where the values come from: the MFMA rows and the VALU -> MFMA / store rows are what hipcc's hazard
recognizer inserts for the same pairs (probed when the generators were written); the rows added in
round 6 are those of LLVM's GCNHazardRecognizer for gfx940/gfx950, each confirmed where a probe can
show it (hipcc -S of a kernel forcing the pair: `v_mad_u64_u32 v0 ...; s_nop 0; v_readfirstlane_b32
s0, v0`, `v_readfirstlane_b32 s0, v3; s_nop 1; v_writelane_b32 v28, s0, 7`, `v_cmp_* vcc; s_nop 1;
v_cndmask_* vcc`). Round 5's wrong results came from the first of these (a `v_readfirstlane` right
after the VALU write of its source returned the old value) — a pair the generators' table did not
hold, since it sat across a statement boundary.
"""

# MFMA D write -> later read of those VGPRs/AGPRs, by the writing MFMA's form:
#   srcc: as srcC of an MFMA; srcab: as srcA / srcB; valu: by a VALU (incl. v_readlane / readfirstlane);
#   vmem: as the data of a VMEM / LDS store
#   (the generators' values; MFMA_HW: where the hardware needs fewer — hipcc's own padding, and
#   srcc_same: srcC exactly the previous D of the same form, the accumulation chain)
MFMA = {
    "v_mfma_f64_4x4x4_4b_f64": dict(srcc=4, srcab=6, valu=6, vmem=10),   # 4 passes
    "v_mfma_f32_16x16x4_f32": dict(srcc=2, srcab=12, valu=12, vmem=12),   # 8 passes (XDL)
}
MFMA_HW = {
    "v_mfma_f64_4x4x4_4b_f64": dict(srcc=4, srcc_same=4, srcab=6, valu=6, vmem=9),
    "v_mfma_f32_16x16x4_f32": dict(srcc=2, srcc_same=0, srcab=10, valu=10, vmem=10),
}
MFMA_DEFAULT = dict(srcc=18, srcc_same=18, srcab=18, valu=18, vmem=18)  # any other form: the 16-pass values

VALU_TO_MFMA = 2           # VALU write VGPR -> MFMA reads it (srcA / srcB / srcC)
VALU_TO_STORE = 2          # VALU write VGPR -> VMEM store reads it as data (generators' margin; hardware: 0)
STORE_WAR = 2              # VMEM store reads VGPRs as data -> a VALU / MFMA / load overwrites them
STORE_WAR_HW = 1           #   (hardware: 1, and only for stores of more than 8 bytes of data)
M0_TO_LDS_DMA = 1          # SALU write M0 -> LDS-DMA (global_load_lds_*, buffer_load_* ... lds)
VALU_VGPR_TO_READLANE = 1  # VALU write VGPR -> v_readlane / v_readfirstlane / v_writelane reads it
VALU_SGPR_TO_VMEM = 5      # VALU write SGPR / VCC (v_readfirstlane, v_cmp, carry-out) -> VMEM reads it
VALU_SGPR_TO_VALU = 2      # VALU write SGPR / VCC -> VALU reads it (constant, carry-in, mask)
VALU_SGPR_TO_LANESEL = 4   # VALU write SGPR -> v_readlane / v_writelane lane select
VALU_VGPR_TO_DPP = 2       # VALU write VGPR -> DPP VALU reads it
GPR_IDX_ON_TO_VALU = 1     # s_set_gpr_idx_on -> the first VALU it indexes (hipcc emits none; the generators pad 1)

# the generators' historic names (gen_chain_asm.py / gen_chain32_asm.py)
F64 = MFMA["v_mfma_f64_4x4x4_4b_f64"]
F32 = MFMA["v_mfma_f32_16x16x4_f32"]
