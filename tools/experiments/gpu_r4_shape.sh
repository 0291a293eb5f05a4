#!/bin/bash
# Round-4 shape A/B: chain microbenchmark (UB), parity (TESTS, PYTEST_ARGS), the bench alternating
# ShapeW4 / ShapeW8 (BENCH, BENCH_ARGS), the 2-rank dist worker with verbose output (DISTDBG).
# Each GPU step has its own limit; the first failure ends it.
set -o pipefail
TAG=${1:-r4shape}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${UB:-1}" = 1 ]; then
  timeout -k 10 300 ./tools/ubench/chain2_bench 96 > $OUT/chain2.txt 2>&1 || { echo "ubench failed"; tail -20 $OUT/chain2.txt; exit 1; }
  cat $OUT/chain2.txt
fi
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest -q -x -m gpu --timeout 120 --timeout-method thread ${PYTEST_ARGS:-tests} > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
if [ "${BENCH:-1}" = 1 ]; then
  for r in 1 2; do
    for sh in ${SHAPES:-w4 w8}; do
      TQR_FLOW_SHAPE=$sh timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-api ${BENCH_ARGS:-} > $OUT/bench_${sh}_$r.json 2> $OUT/bench_${sh}_$r.err || { echo "bench $sh failed"; tail -20 $OUT/bench_${sh}_$r.err; exit 1; }
      python -c "import json,sys; d=json.load(open('$OUT/bench_${sh}_$r.json')); print('$sh', d['ms_per_step'], d['value'], d['roofline']['frac'])"
    done
  done
fi
if [ "${DISTDBG:-0}" = 1 ]; then
  TQR_DIST_VERBOSE=1 TQR_FLOW_GRID=96 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29517 tests/dist_worker.py 1024 1024 128 f64 0 gather > $OUT/distdbg.log 2>&1; echo "dist worker exit $?"; grep -v "^W10\|amdgpu.ids" $OUT/distdbg.log | tail -40
fi
