#!/bin/bash
# fp32 c5 tail after the asm chain: one-element segments (with the lookahead UNMQR alone) in the last
# 32 / 48 steps of 128 against none (the fp32 default), variants alternating.
set -o pipefail
O=gpurun_out/${1:-tail32}
mkdir -p $O
export TMPDIR=/tmp
BENCH_ARGS="--no-single-leg --storage f32 --rows 32768 --cols 32768" bash tools/ab_bench.sh $O/f32 3 libtqr.so libtqr.so:TQR_TAIL=32 libtqr.so:TQR_TAIL=48 libtqr.so:TQR_TAIL=16 || exit 1
