#!/bin/bash
# Panel / lookahead keying re-measured on the final code: fp32 TQR_LA 2 (default) / 4 / 6, fp64
# TQR_LAC 2 / 4 (one GPU; default 0), variants alternating.
set -o pipefail
O=gpurun_out/${1:-la5}
mkdir -p $O
export TMPDIR=/tmp
BENCH_ARGS="--no-single-leg --storage f32 --rows 32768 --cols 32768" bash tools/ab_bench.sh $O/f32 3 libtqr.so libtqr.so:TQR_LA=4 libtqr.so:TQR_LA=6 || exit 1
BENCH_ARGS="--no-single-leg" bash tools/ab_bench.sh $O/f64 3 libtqr.so libtqr.so:TQR_LAC=2 libtqr.so:TQR_LAC=4 || exit 1
