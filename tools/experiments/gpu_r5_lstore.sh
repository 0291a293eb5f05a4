#!/bin/bash
# fp64 late-store hand-over variant (TQR_CHAIN_LSTORE=1: the hand-over stores row pairs < 16, the next
# element's first body the others right before loading the new pairs): parity, then A/B on c3.
set -o pipefail
O=gpurun_out/${1:-lstore}
mkdir -p $O
export TMPDIR=/tmp
TQR_CHAIN_LSTORE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_factor.py -x -q --timeout 300 --timeout-method thread \
  -k "test_factor_vs_oracle or structured or c2 or config_c3" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
BENCH_ARGS="--no-single-leg" bash tools/ab_bench.sh $O/f64 3 libtqr.so libtqr.so:TQR_CHAIN_LSTORE=1 || exit 1
