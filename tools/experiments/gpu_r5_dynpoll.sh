#!/bin/bash
# fp64 asm chain: the first wave to reach each group's sync point does the dependency polls (LDS
# arrival counter; TQR_CA_DYNPOLL) instead of the fixed poll wave: parity of the variant, then A/B.
set -o pipefail
O=gpurun_out/${1:-dynpoll}
mkdir -p $O
export TMPDIR=/tmp
TQR_LIB=libtqr_dynpoll.so timeout -k 10 600 python -u -m pytest tests/test_gpu_factor.py -x -v --timeout 300 --timeout-method thread \
  -k "test_factor_vs_oracle or structured or c2 or chain_forms" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
BENCH_ARGS="--no-single-leg" bash tools/ab_bench.sh $O/f64 3 libtqr.so libtqr_dynpoll.so || exit 1
