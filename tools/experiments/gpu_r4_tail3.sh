#!/bin/bash
# Round 4: fp64 tail segments as the default (engine.hip default_tail) — full parity suite, then
# A/B against TQR_TAIL=0 on c3.
set -o pipefail
OUT=gpurun_out/${1:-r4tail3}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -q -x -m gpu --timeout 120 --timeout-method thread tests > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
bash tools/ab_bench.sh $OUT/ab_f64 3 libtqr.so libtqr.so:TQR_TAIL=0 || exit 1
