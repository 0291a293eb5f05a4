#!/bin/bash
# Round 4: chain segment length on one GPU for the fp32 c5 line (and c3), alternating.
set -o pipefail
OUT=gpurun_out/${1:-r4seg32}
mkdir -p $OUT
for r in 1 2; do
  for sl in 8 12 16 6; do
    TQR_SEGLEN=$sl timeout -k 10 300 python bench.py --storage f32 --rows 32768 --cols 32768 --steps 3 --warmup 1 --no-cpu-baseline --no-host-api > $OUT/c5_sl${sl}_$r.json 2> $OUT/c5_sl${sl}_$r.err || { echo "c5 sl $sl failed"; exit 1; }
    python -c "import json;d=json.load(open('$OUT/c5_sl${sl}_$r.json'));print('c5 seglen $sl', d['ms_per_step'])"
  done
done
for sl in 8 12 16; do
  TQR_SEGLEN=$sl timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-api > $OUT/c3_sl$sl.json 2> $OUT/c3_sl$sl.err || { echo "c3 sl $sl failed"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c3_sl$sl.json'));print('c3 seglen $sl', d['ms_per_step'])"
done
