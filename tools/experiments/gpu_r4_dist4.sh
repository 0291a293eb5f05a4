#!/bin/bash
# Round 4: multi-GPU parity (tests/test_dist.py) and the 2- and 4-rank one-GPU rehearsals of
# 65536x16384 (segment length by world size; the 4-rank one also at TQR_SEGLEN=8).
set -o pipefail
OUT=gpurun_out/${1:-r4dist4}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_dist.py -m gpu -x -v --timeout 560 --timeout-method thread > $OUT/test_dist.log 2>&1 || { echo "test_dist failed"; tail -30 $OUT/test_dist.log; exit 1; }
tail -2 $OUT/test_dist.log
for n in 2 4; do
  TQR_BENCH_DEVICE=0 TQR_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus $n --steps 3 --warmup 1 --no-cpu-baseline --no-host-api > $OUT/r${n}.json 2> $OUT/r${n}.err || { echo "rehearsal $n failed"; tail -5 $OUT/r${n}.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/r${n}.json'));s=d['strong_scaling'];print('$n ranks', d['ms_per_step'], 'seglen', d['config']['chain_segment_length'], 't1', s['t1_ms'], 'speedup', s['speedup'], [r['status'] for r in d['dist']['ranks']])"
done
TQR_SEGLEN=8 TQR_BENCH_DEVICE=0 TQR_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 4 --steps 3 --warmup 1 --no-cpu-baseline --no-host-api > $OUT/r4_sl8.json 2> $OUT/r4_sl8.err || { echo "rehearsal 4 sl8 failed"; exit 1; }
python -c "import json;d=json.load(open('$OUT/r4_sl8.json'));s=d['strong_scaling'];print('4 ranks seglen 8', d['ms_per_step'], 't1', s['t1_ms'], 'speedup', s['speedup'])"
