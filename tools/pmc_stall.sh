#!/bin/bash
# Wave-state PMC pass for the k_flow launch (default 16384^2 fp64; BENCH_ARGS to change): where the
# waves' cycles go — SQ_WAIT_ANY (parked on s_waitcnt / barrier), SQ_WAIT_INST_ANY (issue stalls:
# MFMA pipe busy / dependency), SQ_ACTIVE_INST_* (issuing) — one rocprofv3 --pmc pass (8 SQ slots,
# no trace domains), summarised by tools/pmc_stall.py.
set -o pipefail
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc_stall}
mkdir -p $OUT
PASS=${PASS:-stall}
if [ "$PASS" = lds ]; then CTRS="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"; else CTRS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"; fi
timeout -s KILL 120 rocprofv3 --pmc $CTRS -d $OUT/$PASS -o pmc --output-format csv -- python3 bench.py --no-cpu-baseline --no-host-api --steps 1 --warmup 0 ${BENCH_ARGS:-} > $OUT/$PASS.log 2>&1 || { echo "pmc $PASS pass failed"; tail -20 $OUT/$PASS.log; exit 1; }
python3 tools/pmc_stall.py $OUT $PASS
