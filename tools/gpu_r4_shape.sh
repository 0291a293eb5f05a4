#!/bin/bash
# Round-4 shape A/B: chain microbenchmark, parity on the fp64 default shape (ShapeW4), then the
# 16384^2 bench alternating ShapeW4 / ShapeW8 (TQR_FLOW_SHAPE=w8). First failure ends it.
set -o pipefail
TAG=${1:-r4shape}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${UB:-1}" = 1 ]; then
  timeout -k 10 300 ./tools/ubench/chain2_bench 96 > $OUT/chain2.txt 2>&1 || { echo "ubench failed"; tail -20 $OUT/chain2.txt; exit 1; }
  cat $OUT/chain2.txt
fi
timeout -k 10 900 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread ${PYTEST_ARGS:-tests/test_gpu_factor.py} > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for r in 1 2; do
  for sh in w4 w8; do
    TQR_FLOW_SHAPE=$sh timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-api ${BENCH_ARGS:-} > $OUT/bench_${sh}_$r.json 2> $OUT/bench_${sh}_$r.err || { echo "bench $sh failed"; tail -20 $OUT/bench_${sh}_$r.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$OUT/bench_${sh}_$r.json')); print('$sh', d['ms_per_step'], d['value'], d['roofline']['frac'])"
  done
done
