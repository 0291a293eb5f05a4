#!/bin/bash
# fp32 asm chain: the poll wave (7) at MFMA issue priority 3 in both phases (generator GEN_PWPRIO),
# so it reaches the group barrier with its polls done; A/B on c5.
set -o pipefail
O=gpurun_out/${1:-pwprio}
mkdir -p $O
export TMPDIR=/tmp
BENCH_ARGS="--no-single-leg --storage f32 --rows 32768 --cols 32768" bash tools/ab_bench.sh $O/f32 3 libtqr.so libtqr_pwprio.so || exit 1
