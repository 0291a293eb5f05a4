#!/bin/bash
# Round 4: chain segment length (TQR_SEGLEN) on one GPU (65536x16384, 16384^2) and in the
# 2-rank one-GPU rehearsal of 65536x16384 (tools/sched_sim.py: S(8) 5.39 at 8, 6.31 at 2).
set -o pipefail
OUT=gpurun_out/${1:-r4seg}
mkdir -p $OUT
for sl in 8 2 4; do
  TQR_SEGLEN=$sl timeout -k 10 300 python bench.py --rows 65536 --cols 16384 --steps 3 --warmup 1 --no-cpu-baseline --no-host-api > $OUT/c4_1gpu_sl$sl.json 2> $OUT/c4_1gpu_sl$sl.err || { echo "c4 sl $sl failed"; tail -5 $OUT/c4_1gpu_sl$sl.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c4_1gpu_sl$sl.json'));print('c4 1gpu seglen $sl', d['ms_per_step'])"
done
for sl in 8 2; do
  TQR_SEGLEN=$sl timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-api > $OUT/c3_sl$sl.json 2> $OUT/c3_sl$sl.err || { echo "c3 sl $sl failed"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c3_sl$sl.json'));print('c3 seglen $sl', d['ms_per_step'])"
done
for sl in 8 2; do
  TQR_SEGLEN=$sl TQR_BENCH_DEVICE=0 TQR_BENCH_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-host-api > $OUT/r2_sl$sl.json 2> $OUT/r2_sl$sl.err || { echo "2-rank sl $sl failed"; tail -5 $OUT/r2_sl$sl.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/r2_sl$sl.json'));s=d['strong_scaling'];print('2-rank seglen $sl', d['ms_per_step'], 't1', s['t1_ms'], 'speedup', s['speedup'])"
done
