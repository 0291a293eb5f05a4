#!/bin/bash
# fp64 GEQRT trailing update over the k-steps below the group only (and fp64 XLEAD 2): parity, then
# A/B against the full-V trailing update (libtqr_gefull.so, -DTQR_PANEL_GE_FULL).
set -o pipefail
O=gpurun_out/${1:-gepanel}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_factor.py -x -v --timeout 300 --timeout-method thread \
  -k "test_factor_vs_oracle or structured or zero_row or c2 or chain_knobs or chain_forms" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
BENCH_ARGS="--no-single-leg" bash tools/ab_bench.sh $O/ab 3 libtqr.so libtqr_gefull.so || exit 1
