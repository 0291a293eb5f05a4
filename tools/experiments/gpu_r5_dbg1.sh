#!/bin/bash
# Isolate: (1) the fp32 asm chain and the lookahead UNMQR-alone segment on single-GPU parity tests,
# (2) the 2-rank dist test with / without TQR_UNMQR_ALONE.
set -o pipefail
O=gpurun_out/${1:-dbg1}
mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
TQR_UNMQR_ALONE=0 TQR_CHAIN32_ASM=0 timeout -k 10 300 $T tests/test_gpu_factor.py -k "test_factor_vs_oracle" > $O/base.log 2>&1; echo "base rc=$?"; tail -3 $O/base.log
TQR_CHAIN32_ASM=0 timeout -k 10 300 $T tests/test_gpu_factor.py -k "test_factor_vs_oracle" > $O/ualone.log 2>&1; echo "ualone rc=$?"; tail -3 $O/ualone.log
TQR_UNMQR_ALONE=0 timeout -k 10 300 $T tests/test_gpu_factor.py -k "test_factor_vs_oracle" > $O/asm32.log 2>&1; echo "asm32 rc=$?"; tail -3 $O/asm32.log
