#!/bin/bash
# Round 4: does the fp64 tail rule (<= 31 rows below the diagonal) carry to other sizes?
set -o pipefail
OUT=gpurun_out/${1:-r4tail6}
mkdir -p $OUT
BENCH_ARGS="--rows 8192 --cols 8192" bash tools/ab_bench.sh $OUT/ab_8192 2 libtqr.so libtqr.so:TQR_TAIL=0 || exit 1
BENCH_ARGS="--rows 24576 --cols 24576" bash tools/ab_bench.sh $OUT/ab_24576 2 libtqr.so libtqr.so:TQR_TAIL=0 || exit 1
