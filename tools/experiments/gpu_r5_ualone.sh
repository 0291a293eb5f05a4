#!/bin/bash
# Tail: the lookahead column's UNMQR element alone in segment 0 (TQR_UNMQR_ALONE, default = the
# tail steps): full GPU suite, then A/B against TQR_UNMQR_ALONE=0, then the tail timeline.
set -o pipefail
O=gpurun_out/${1:-ualone}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
BENCH_ARGS="--no-single-leg" bash tools/ab_bench.sh $O/ab 3 libtqr.so libtqr.so:TQR_UNMQR_ALONE=0 || exit 1
TQR_TIMELINE_TAIL=8 timeout -k 10 300 python tools/timeline.py 16384 256 > $O/timeline_f64.txt 2>&1 || { echo "timeline failed"; tail -20 $O/timeline_f64.txt; exit 1; }
head -22 $O/timeline_f64.txt
