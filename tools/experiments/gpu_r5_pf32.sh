#!/bin/bash
# fp32 asm chain: the panel counter prefetch by the wave beside the poll wave (into the poll wave's LDS
# view, as the fp64 chain) against the poll wave's own prefetch (libtqr_pfpw.so): parity, A/B on c5.
set -o pipefail
O=gpurun_out/${1:-pf32}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_factor.py -x -v --timeout 300 --timeout-method thread \
  -k "test_factor_vs_oracle or chain_knobs or fp32" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
BENCH_ARGS="--no-single-leg --storage f32 --rows 32768 --cols 32768" bash tools/ab_bench.sh $O/f32 3 libtqr.so libtqr_pfpw.so || exit 1
