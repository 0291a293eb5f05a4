#!/bin/bash
# Round 4: A/B of the panel variants (TQR_PSPLIT 0 / 1 / 3) and of the chain's poll wave (TQR_CHAIN_PT
# builds) against the round-3 engine (libtqr_base.so), fp64 16384^2 then fp32 32768^2.
set -o pipefail
OUT=gpurun_out/${1:-r4ab2}
mkdir -p $OUT
bash tools/ab_bench.sh $OUT/ab_f64 2 libtqr_base.so libtqr.so:TQR_PSPLIT=0 libtqr.so:TQR_PSPLIT=1 libtqr_pt192.so:TQR_PSPLIT=0 libtqr_pt64.so:TQR_PSPLIT=0 || exit 1
BENCH_ARGS="--storage f32 --rows 32768 --cols 32768" bash tools/ab_bench.sh $OUT/ab_f32 2 libtqr_base.so libtqr.so:TQR_PSPLIT=0 libtqr.so:TQR_PSPLIT=1 || exit 1
