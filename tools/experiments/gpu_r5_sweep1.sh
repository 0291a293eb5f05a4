#!/bin/bash
# Knob sweep after the fp32 asm chain and the tail change (one call, variants alternating):
# fp32 c5: late-load lead (generator XLEAD 4 / 6 / 8), tail steps, panel lookahead, segment length;
# fp64 c3: the UNMQR-alone segments on more steps.
set -o pipefail
O=gpurun_out/${1:-sweep1}
mkdir -p $O
export TMPDIR=/tmp
BENCH_ARGS="--no-single-leg --storage f32 --rows 32768 --cols 32768" bash tools/ab_bench.sh $O/f32 2 libtqr.so libtqr_xl4.so libtqr_xl8.so \
  libtqr.so:TQR_TAIL=16 libtqr.so:TQR_TAIL=32 libtqr.so:TQR_LA=0 libtqr.so:TQR_LA=4 libtqr.so:TQR_SEGLEN=6 libtqr.so:TQR_SEGLEN=12 || exit 1
BENCH_ARGS="--no-single-leg" bash tools/ab_bench.sh $O/f64 2 libtqr.so libtqr.so:TQR_UNMQR_ALONE=64 \
  libtqr.so:TQR_TAIL=40,TQR_UNMQR_ALONE=40 libtqr.so:TQR_TAIL=24,TQR_UNMQR_ALONE=24 || exit 1
