#!/bin/bash
# Round 4: tail segment-length sweep, second pass (longer tails, two-element tail segments).
set -o pipefail
OUT=gpurun_out/${1:-r4tail2}
mkdir -p $OUT
bash tools/ab_bench.sh $OUT/ab_f64 2 libtqr.so:TQR_TAIL=24 libtqr.so:TQR_TAIL=32 libtqr.so:TQR_TAIL=40 libtqr.so:TQR_TAIL=48 libtqr.so:TQR_TAIL=32,TQR_TAIL_SEGLEN=2 libtqr.so:TQR_TAIL=48,TQR_TAIL_SEGLEN=2 || exit 1
BENCH_ARGS="--storage f32 --rows 32768 --cols 32768" bash tools/ab_bench.sh $OUT/ab_f32 1 libtqr.so libtqr.so:TQR_TAIL=48 libtqr.so:TQR_TAIL=64 libtqr.so:TQR_TAIL=96 libtqr.so:TQR_TAIL=64,TQR_TAIL_SEGLEN=2 || exit 1
