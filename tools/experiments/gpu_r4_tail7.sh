#!/bin/bash
# Round 4: fp32 storage, one-element segments in the very last steps only.
set -o pipefail
OUT=gpurun_out/${1:-r4tail7}
mkdir -p $OUT
BENCH_ARGS="--storage f32 --rows 32768 --cols 32768" bash tools/ab_bench.sh $OUT/ab_f32 2 libtqr.so libtqr.so:TQR_TAIL=4 libtqr.so:TQR_TAIL=8 libtqr.so:TQR_TAIL=8,TQR_TAIL_SEGLEN=2 || exit 1
