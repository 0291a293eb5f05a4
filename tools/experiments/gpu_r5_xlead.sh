#!/bin/bash
# Late-load lead in the engine: fp64 XLEAD 2 / 4 (default) / 6 / 8 row pairs, fp32 XLEAD 5 / 6 (default)
# / 7 tiles (generator variants built with TQR_C64_INC / TQR_C32_INC), variants alternating.
set -o pipefail
O=gpurun_out/${1:-xlead}
mkdir -p $O
export TMPDIR=/tmp
BENCH_ARGS="--no-single-leg" bash tools/ab_bench.sh $O/f64 3 libtqr.so libtqr_f64xl2.so libtqr_f64xl6.so libtqr_f64xl8.so || exit 1
BENCH_ARGS="--no-single-leg --storage f32 --rows 32768 --cols 32768" bash tools/ab_bench.sh $O/f32 2 libtqr.so libtqr_f32xl5.so libtqr_f32xl7.so || exit 1
