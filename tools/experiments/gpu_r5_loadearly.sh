#!/bin/bash
# Panel members load their own block before waiting for the previous member's R rows (Rr): parity,
# then A/B against the block loaded after the wait (libtqr_loadlate.so), c3 fp64 and c5 fp32.
set -o pipefail
O=gpurun_out/${1:-loadearly}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_factor.py tests/test_dist.py -x -q --timeout 300 --timeout-method thread \
  -k "test_factor_vs_oracle or structured or zero_row or c2 or chain_knobs or ranks_on_one_gpu and not 65536" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
BENCH_ARGS="--no-single-leg" bash tools/ab_bench.sh $O/f64 3 libtqr.so libtqr_loadlate.so || exit 1
BENCH_ARGS="--no-single-leg --storage f32 --rows 32768 --cols 32768" bash tools/ab_bench.sh $O/f32 2 libtqr.so libtqr_loadlate.so || exit 1
