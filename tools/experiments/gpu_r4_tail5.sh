#!/bin/bash
# Round 4: with the fp64 tail segments, the lookahead column's segment length in the other steps.
set -o pipefail
OUT=gpurun_out/${1:-r4tail5}
mkdir -p $OUT
bash tools/ab_bench.sh $OUT/ab_f64 2 libtqr.so libtqr.so:TQR_SEGLEN_LA=4 libtqr.so:TQR_SEGLEN_LA=2 libtqr.so:TQR_SEGLEN_LA=1 || exit 1
