#!/bin/bash
# Round 4: f_j without the reciprocal of hd (panel_step) — ubench, parity, A/B c3 / c5.
set -o pipefail
OUT=gpurun_out/${1:-r4fm}
mkdir -p $OUT
timeout -k 10 120 ./tools/ubench/panel_bench_fm > $OUT/panel_bench_fm.txt 2>&1 || { echo "ubench failed"; exit 1; }
timeout -k 10 120 ./tools/ubench/panel_bench_w8 > $OUT/panel_bench_base.txt 2>&1 || exit 1
head -8 $OUT/panel_bench_fm.txt; head -8 $OUT/panel_bench_base.txt
timeout -k 10 900 python -u -m pytest -q -x -m gpu --timeout 120 --timeout-method thread tests > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
bash tools/ab_bench.sh $OUT/ab_f64 2 libtqr_base.so libtqr.so || exit 1
BENCH_ARGS="--storage f32 --rows 32768 --cols 32768" bash tools/ab_bench.sh $OUT/ab_f32 2 libtqr_base.so libtqr.so || exit 1
