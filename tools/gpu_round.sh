#!/bin/bash
# One GPU-box pass: parity tests, bench, engine activity stamps, rocprofv3 kernel-trace summary.
# Each GPU step has its own time limit; the first failure ends the script (no retries).
# Outputs under gpurun_out/$TAG. Env: TESTS=0 skips pytest, PROF=0 skips rocprof, FST=0 skips stamps.
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
if [ "${FST:-1}" = 1 ] && [ -f gpu-tiled-qr-decomposition_amd/libtqr_fst.so ]; then
  timeout -k 10 120 python tools/flowstamps.py 16384 > $OUT/flowstamps.txt 2>&1 || { echo "flowstamps failed"; tail -20 $OUT/flowstamps.txt; exit 1; }
  grep -v amdgpu.ids $OUT/flowstamps.txt
  timeout -k 10 120 python tools/timeline.py 16384 > $OUT/timeline.txt 2>&1 || { echo "timeline failed"; tail -20 $OUT/timeline.txt; exit 1; }
  grep -v amdgpu.ids $OUT/timeline.txt
  timeout -k 10 120 python tools/group_trace.py 16384 > $OUT/group_trace.txt 2>&1 || { echo "group_trace failed"; tail -20 $OUT/group_trace.txt; exit 1; }
  grep -v amdgpu.ids $OUT/group_trace.txt
fi
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
  find $OUT/prof -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200
fi
