#!/bin/bash
# Round 4 split panel trailing: parity (TESTS), activity stamps (FST), A/B against the previous
# engine (AB: libtqr_base.so vs libtqr.so, fp64 16384^2 and fp32 32768^2). First failure ends it.
set -o pipefail
TAG=${1:-r4split}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest -q -x -m gpu --timeout 120 --timeout-method thread ${PYTEST_ARGS:-tests} > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
if [ "${FST:-1}" = 1 ]; then
  timeout -k 10 120 python tools/flowstamps.py 16384 > $OUT/flowstamps_f64.txt 2>&1 || { echo "flowstamps failed"; tail -20 $OUT/flowstamps_f64.txt; exit 1; }
  head -8 $OUT/flowstamps_f64.txt
  TQR_FST_DTYPE=f32 timeout -k 10 180 python tools/flowstamps.py 32768 > $OUT/flowstamps_f32.txt 2>&1 || { echo "flowstamps f32 failed"; tail -20 $OUT/flowstamps_f32.txt; exit 1; }
  head -8 $OUT/flowstamps_f32.txt
fi
if [ "${AB:-1}" = 1 ]; then
  bash tools/ab_bench.sh $OUT/ab_f64 2 libtqr_base.so libtqr.so || exit 1
  BENCH_ARGS="--storage f32 --rows 32768 --cols 32768" bash tools/ab_bench.sh $OUT/ab_f32 2 libtqr_base.so libtqr.so || exit 1
fi
