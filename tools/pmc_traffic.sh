#!/bin/bash
# PMC evidence for one k_flow launch (default 16384^2, b=256; BENCH_ARGS to change): three
# rocprofv3 --pmc passes (counters kept within one pass's slots, no trace domains), then
# tools/pmc_summary.py writes profiles/pmc_summary.json:
#   FETCH_SIZE | WRITE_SIZE                       HBM-side bytes (gfx950 FETCH_SIZE x2 correction)
#   SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
#                                                 executed MFMA flops and MFMA-pipe utilisation
# Output CSVs under gpurun_out/pmc/<pass>/ (copy to profiles/ to keep them).
set -o pipefail
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc}
mkdir -p $OUT
run_pass() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $OUT/$name -o pmc --output-format csv -- python3 bench.py --no-cpu-baseline --no-host-api --steps 1 --warmup 1 ${BENCH_ARGS:-} > $OUT/$name.log 2>&1 || { echo "pmc pass $name failed"; tail -20 $OUT/$name.log; exit 1; }
}
run_pass FETCH_SIZE FETCH_SIZE
run_pass WRITE_SIZE WRITE_SIZE
run_pass MFMA SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
python3 tools/pmc_summary.py $OUT ${PMC_KEY:-}
