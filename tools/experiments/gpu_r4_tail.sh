#!/bin/bash
# Round 4: chains of the last TQR_TAIL steps one element per segment — parity with the knob set,
# then A/B on c3 / c5 against the default list.
set -o pipefail
OUT=gpurun_out/${1:-r4tail}
mkdir -p $OUT
TQR_TAIL=16 timeout -k 10 600 python -u -m pytest -q -x -m gpu --timeout 120 --timeout-method thread tests/test_gpu_factor.py tests/test_gpu_xfer.py > $OUT/pytest_gpu_tail16.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu_tail16.log; exit 1; }
tail -1 $OUT/pytest_gpu_tail16.log
bash tools/ab_bench.sh $OUT/ab_f64 2 libtqr.so libtqr.so:TQR_TAIL=8 libtqr.so:TQR_TAIL=16 libtqr.so:TQR_TAIL=24 || exit 1
BENCH_ARGS="--storage f32 --rows 32768 --cols 32768" bash tools/ab_bench.sh $OUT/ab_f32 2 libtqr.so libtqr.so:TQR_TAIL=16 libtqr.so:TQR_TAIL=32 || exit 1
