#!/bin/bash
# One GPU-box pass: parity tests, bench, rocprofv3 kernel-trace summary. Each GPU step has its
# own time limit; the first failure ends the script (no retries). Outputs under gpurun_out/$TAG.
set -o pipefail
TAG=${1:-run}
TESTS=${TESTS:-1}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$TESTS" = 1 ]; then
  timeout -k 10 600 python -m pytest tests -q -x -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
  find $OUT/prof -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200
fi
