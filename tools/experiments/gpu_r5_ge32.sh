#!/bin/bash
# fp32 UNMQR element skipping the GE V's zero tiles (apply32 K0 = g NMI): full GPU suite, then
# A/B on c5 against the build without the skip (libtqr_noge32.so, -DTQR_NO_GE_SKIP32).
set -o pipefail
O=gpurun_out/${1:-ge32}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
BENCH_ARGS="--no-single-leg --storage f32 --rows 32768 --cols 32768" bash tools/ab_bench.sh $O/ab 3 libtqr.so libtqr_noge32.so
