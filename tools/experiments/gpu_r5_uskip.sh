#!/bin/bash
# UNMQR elements on bodies that skip the GE V's zero rows (group g: k-steps >= 8 g) and store the
# finished rows group by group: parity (both hand-over forms), then A/B against TQR_UNMQR_SKIP=0.
set -o pipefail
O=gpurun_out/${1:-uskip}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_factor.py -x -v --timeout 300 --timeout-method thread \
  -k "test_factor_vs_oracle or structured or zero_row or full_size or c2 or chain_forms" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
BENCH_ARGS="--no-cpu-baseline --no-host-api --no-single-leg" bash tools/ab_bench.sh $O/ab 3 libtqr.so:TQR_UNMQR_SKIP=1 libtqr.so:TQR_UNMQR_SKIP=0
