#!/bin/bash
# Parity of the lookahead UNMQR-alone segments (fp64 tail) and the fp32 asm chain (full suite),
# then A/B: fp64 c3 against TQR_UNMQR_ALONE=0, fp32 c5 against TQR_CHAIN32_ASM=0.
set -o pipefail
O=gpurun_out/${1:-ab2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_factor.py -x -v --timeout 200 --timeout-method thread -k "test_factor_vs_oracle" > $O/quick.log 2>&1 || { echo "quick parity failed"; tail -30 $O/quick.log; exit 1; }
tail -2 $O/quick.log
timeout -k 10 700 python -u -m pytest tests -q -x -m gpu --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
BENCH_ARGS="--no-single-leg" bash tools/ab_bench.sh $O/ab64 3 libtqr.so libtqr.so:TQR_UNMQR_ALONE=0 || exit 1
BENCH_ARGS="--no-single-leg --storage f32 --rows 32768 --cols 32768" bash tools/ab_bench.sh $O/ab32 2 libtqr.so libtqr.so:TQR_CHAIN32_ASM=0 || exit 1
