#!/bin/bash
# fp64 asm chain: the poll wave (7) at MFMA issue priority 3 in both phases (GEN_PWPRIO); A/B on c3.
set -o pipefail
O=gpurun_out/${1:-pwprio64}
mkdir -p $O
export TMPDIR=/tmp
BENCH_ARGS="--no-single-leg" bash tools/ab_bench.sh $O/f64 3 libtqr.so libtqr_pwprio64.so || exit 1
