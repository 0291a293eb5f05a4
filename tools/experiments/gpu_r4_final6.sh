#!/bin/bash
# Round 4 (late): final evidence with the fp32 lookahead default, then its A/B against TQR_LA=0.
set -o pipefail
bash tools/gpu_final.sh ${1:-r4final6} || exit 1
BENCH_ARGS="--storage f32 --rows 32768 --cols 32768" bash tools/ab_bench.sh gpurun_out/${1:-r4final6}/ab_f32_la 2 libtqr.so libtqr.so:TQR_LA=0 || exit 1
