#!/bin/bash
# Round 4: around the fp64 default tail — other tail lengths and body segment lengths with it.
set -o pipefail
OUT=gpurun_out/${1:-r4tail4}
mkdir -p $OUT
bash tools/ab_bench.sh $OUT/ab_f64 2 libtqr.so libtqr.so:TQR_TAIL=28 libtqr.so:TQR_TAIL=36 libtqr.so:TQR_SEGLEN=6 libtqr.so:TQR_SEGLEN=4 libtqr.so:TQR_SEGLEN=12 || exit 1
