#!/bin/bash
# Panel write-back split around the Rr publish (R rows first, V rows and tau after): parity, then
# A/B against the whole block before the publish (libtqr_wbwhole.so), fp64 c3 and fp32 c5.
set -o pipefail
O=gpurun_out/${1:-wb}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_factor.py -x -v --timeout 300 --timeout-method thread \
  -k "test_factor_vs_oracle or structured or zero_row or c2 or chain_knobs" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
BENCH_ARGS="--no-single-leg" bash tools/ab_bench.sh $O/f64 3 libtqr.so libtqr_wbwhole.so || exit 1
BENCH_ARGS="--no-single-leg --storage f32 --rows 32768 --cols 32768" bash tools/ab_bench.sh $O/f32 2 libtqr.so libtqr_wbwhole.so || exit 1
