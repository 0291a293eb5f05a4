#!/bin/bash
# fp64 c3 segment length after the asm chain (8 default; 6 / 10 / 12), variants alternating.
set -o pipefail
O=gpurun_out/${1:-seg64}
mkdir -p $O
export TMPDIR=/tmp
BENCH_ARGS="--no-single-leg" bash tools/ab_bench.sh $O/f64 3 libtqr.so libtqr.so:TQR_SEGLEN=6 libtqr.so:TQR_SEGLEN=10 libtqr.so:TQR_SEGLEN=12 || exit 1
