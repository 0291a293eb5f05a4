#!/bin/bash
# Round 5, first look at the hand-scheduled fp64 chain: factorisation parity, then an A/B of the
# asm chain against the compiler-scheduled one (TQR_CHAIN_ASM=0) at 16384^2.
set -o pipefail
O=gpurun_out/${1:-r5a}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_factor.py -x -v --timeout 120 --timeout-method thread > $O/pytest_factor.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_factor.log; exit 1; }
tail -3 $O/pytest_factor.log
bash tools/ab_bench.sh $O/ab 2 libtqr.so:TQR_CHAIN_ASM=1 libtqr.so:TQR_CHAIN_ASM=0
