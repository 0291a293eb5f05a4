#!/bin/bash
# fp64 late-load lead around the new default: XLEAD 1 / 2 (default) / 3 row pairs; parity of the
# variants, then A/B on c3.
set -o pipefail
O=gpurun_out/${1:-xlead2}
mkdir -p $O
export TMPDIR=/tmp
for L in libtqr_f64xl1.so libtqr_f64xl3.so; do
  TQR_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_factor.py -x -q --timeout 300 --timeout-method thread \
    -k "test_factor_vs_oracle or c2 or chain_forms" > $O/pytest_$L.log 2>&1 || { echo "pytest $L failed"; tail -30 $O/pytest_$L.log; exit 1; }
  tail -1 $O/pytest_$L.log
done
BENCH_ARGS="--no-single-leg" bash tools/ab_bench.sh $O/f64 3 libtqr.so libtqr_f64xl1.so libtqr_f64xl3.so || exit 1
