#!/bin/bash
# Round-4 GPU pass: parity suite, default bench, and the plain (self-launching) 2-rank rehearsal
# of bench.py --gpus 2 on one GPU. Each GPU step has its own limit; the first failure ends it.
set -o pipefail
TAG=${1:-r4}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -20 $OUT/bench_default.err; exit 1; }
  cat $OUT/bench_default.json
fi
if [ "${DIST:-1}" = 1 ]; then
  TQR_BENCH_DEVICE=0 TQR_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 3 --warmup 1 --rows 32768 --cols 8192 > $OUT/bench_gpus2.json 2> $OUT/bench_gpus2.err || { echo "bench --gpus 2 failed"; tail -30 $OUT/bench_gpus2.err; exit 1; }
  cat $OUT/bench_gpus2.json
fi
