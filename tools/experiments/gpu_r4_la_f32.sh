#!/bin/bash
# Round 4 (late): fp32 panel lookahead keying (TQR_LA, chain elements) re-measured on the final code.
set -o pipefail
OUT=gpurun_out/${1:-r4laf32}
mkdir -p $OUT
BENCH_ARGS="--storage f32 --rows 32768 --cols 32768" bash tools/ab_bench.sh $OUT/ab_f32 2 libtqr.so libtqr.so:TQR_LA=2 libtqr.so:TQR_LA=4 libtqr.so:TQR_LA=6 || exit 1
bash tools/ab_bench.sh $OUT/ab_f64 2 libtqr.so libtqr.so:TQR_LA=2 libtqr.so:TQR_LA=4 || exit 1
