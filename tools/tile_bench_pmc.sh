#!/bin/bash
# PMC evidence for the per-tile-op microbench: the tools/tile_bench.py sweep
# (fp64/fp32 x b = 16..256 x TSMQR/UNMQR, 3 launches of k_update each) under three rocprofv3
# --pmc passes (counters within one pass's slots, no trace domains), then
# tools/tile_bench_pmc.py joins each configuration's last launch with its JSON line:
# MFMA-pipe utilisation, executed vs algorithmic flops, HBM bytes (FETCH_SIZE x2 + WRITE_SIZE).
set -o pipefail
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/tile_pmc}
mkdir -p $OUT
run_pass() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 180 rocprofv3 --pmc "$@" -d $OUT/$name -o pmc --output-format csv -- python3 tools/tile_bench.py > $OUT/$name.jsonl 2> $OUT/$name.log || { echo "pmc pass $name failed"; tail -20 $OUT/$name.log; exit 1; }
}
run_pass FETCH_SIZE FETCH_SIZE
run_pass WRITE_SIZE WRITE_SIZE
run_pass MFMA SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
python3 tools/tile_bench_pmc.py $OUT > $OUT/tile_bench_pmc.jsonl
cat $OUT/tile_bench_pmc.jsonl
