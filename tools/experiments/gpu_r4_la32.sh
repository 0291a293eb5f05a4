#!/bin/bash
# Round 4: panel-first list keys (TQR_LA, chain elements) for the fp32 c5 line, alternating.
set -o pipefail
OUT=gpurun_out/${1:-r4la32}
mkdir -p $OUT
for r in 1 2; do
  for la in 0 4 10 25; do
    TQR_LA=$la TQR_LAC=0 timeout -k 10 300 python bench.py --storage f32 --rows 32768 --cols 32768 --steps 3 --warmup 1 --no-cpu-baseline --no-host-api > $OUT/c5_la${la}_$r.json 2> $OUT/c5_la${la}_$r.err || { echo "c5 la $la failed"; exit 1; }
    python -c "import json;d=json.load(open('$OUT/c5_la${la}_$r.json'));print('c5 TQR_LA $la', d['ms_per_step'])"
  done
done
