#!/bin/bash
# Round-end evidence pass on one GPU box: parity suite, default bench (fp64 16384^2, with
# cpu_baseline and host_api), the fp32 32768^2 line (with its fp32 cpu_baseline), rocprofv3
# kernel-trace summaries of both, and optionally the PMC passes (PMC=1).
# Usage: bash tools/gpu_final.sh TAG. Each GPU step has its own limit; the first failure ends it.
set -o pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 700 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -20 $OUT/bench_default.err; exit 1; }
  cat $OUT/bench_default.json
  timeout -k 10 400 python bench.py --storage f32 --rows 32768 --cols 32768 > $OUT/bench_f32_c5.json 2> $OUT/bench_f32_c5.err || { echo "bench f32 failed"; tail -20 $OUT/bench_f32_c5.err; exit 1; }
  cat $OUT/bench_f32_c5.json
fi
if [ "${C4:-0}" = 1 ]; then  # the 65536 x 16384 one-GPU line (the multi-GPU model's calibration)
  timeout -k 10 300 python bench.py --rows 65536 --cols 16384 --no-cpu-baseline --no-host-api > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { echo "bench c4 failed"; tail -20 $OUT/bench_c4.err; exit 1; }
  cat $OUT/bench_c4.json
fi
if [ "${TIMELINE:-0}" = 1 ]; then  # the last steps' task timeline (stamps build libtqr_fst.so)
  TQR_TIMELINE_TAIL=8 timeout -k 10 300 python tools/timeline.py 16384 256 > $OUT/timeline_f64.txt 2>&1 || { echo "timeline failed"; tail -20 $OUT/timeline_f64.txt; exit 1; }
  head -24 $OUT/timeline_f64.txt
fi
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_f64 -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-host-api --steps 3 --warmup 1 > $OUT/prof_f64.log 2>&1 || { echo "rocprof f64 failed"; tail -20 $OUT/prof_f64.log; exit 1; }
  find $OUT/prof_f64 -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200 | head -5
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_f32 -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-host-api --storage f32 --rows 32768 --cols 32768 --steps 2 --warmup 1 > $OUT/prof_f32.log 2>&1 || { echo "rocprof f32 failed"; tail -20 $OUT/prof_f32.log; exit 1; }
  find $OUT/prof_f32 -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200 | head -5
fi
if [ "${PMC:-0}" = 1 ]; then
  PMC_OUT=$OUT/pmc bash tools/pmc_traffic.sh || exit 1
  PMC_OUT=$OUT/pmc_f32 PMC_KEY=32768x32768_b256_f32 BENCH_ARGS="--storage f32 --rows 32768 --cols 32768" bash tools/pmc_traffic.sh || exit 1
fi
