#!/bin/bash
# W8 asm chain with late strip loads (TQR_CHAIN_ASM=2: the hand-over loads only the next strip's first
# XLEAD row pairs, the next element's first body the rest inside its phase 1): parity, then A/B.
set -o pipefail
O=gpurun_out/${1:-late}
mkdir -p $O
export TMPDIR=/tmp
TQR_CHAIN_ASM=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_factor.py -x -v --timeout 300 --timeout-method thread \
  -k "test_factor_vs_oracle or structured or zero_row or full_size or c2" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
BENCH_ARGS="--no-cpu-baseline --no-host-api --no-single-leg" bash tools/ab_bench.sh $O/ab 3 libtqr.so:TQR_CHAIN_ASM=2 libtqr.so:TQR_CHAIN_ASM=1
