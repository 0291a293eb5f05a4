#!/bin/bash
# Task-list order knobs after the round-5 chains (the estimator's panel group cost TQR_TG and the
# lazy keying TQR_LAZY): c3 fp64 and c5 fp32, variants alternating.
set -o pipefail
O=gpurun_out/${1:-order5}
mkdir -p $O
export TMPDIR=/tmp
BENCH_ARGS="--no-single-leg" bash tools/ab_bench.sh $O/f64 2 libtqr.so libtqr.so:TQR_TG=0.6 libtqr.so:TQR_TG=1.0 libtqr.so:TQR_TG=2.0 \
  libtqr.so:TQR_LAZY=0 libtqr.so:TQR_LAZY=0.5 libtqr.so:TQR_LAZY=1.5 || exit 1
BENCH_ARGS="--no-single-leg --storage f32 --rows 32768 --cols 32768" bash tools/ab_bench.sh $O/f32 2 libtqr.so libtqr.so:TQR_TG=1.0 \
  libtqr.so:TQR_TG=2.0 libtqr.so:TQR_LAZY=0.5 libtqr.so:TQR_LAZY=1.5 || exit 1
