#!/bin/bash
# Round 4: the fp32 chain's hand-over flag read as an LDS read (no flat-load drain) — parity of
# the fp32 tests, A/B on c5.
set -o pipefail
OUT=gpurun_out/${1:-r4c32flag}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -q -x -m gpu --timeout 120 --timeout-method thread tests/test_gpu_factor.py > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
BENCH_ARGS="--storage f32 --rows 32768 --cols 32768" bash tools/ab_bench.sh $OUT/ab_f32 2 libtqr_base.so libtqr.so || exit 1
