#!/bin/bash
# Resident-form chain (ShapeR, TQR_FLOW_SHAPE=r): parity on the b = 256 cases and the full-size
# properties, then an A/B against the 8-wave asm chain at 16384^2.
set -o pipefail
O=gpurun_out/${1:-res2}
mkdir -p $O
export TMPDIR=/tmp
TQR_FLOW_SHAPE=r timeout -k 10 600 python -u -m pytest tests/test_gpu_factor.py -x -v --timeout 300 --timeout-method thread \
  -k "(test_factor_vs_oracle and 256 and float64) or structured or zero_row or (full_size and 16384-16384)" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
BENCH_ARGS="--no-cpu-baseline --no-host-api --no-single-leg" bash tools/ab_bench.sh $O/ab 2 libtqr.so:TQR_FLOW_SHAPE=r libtqr.so:TQR_FLOW_SHAPE=w8
