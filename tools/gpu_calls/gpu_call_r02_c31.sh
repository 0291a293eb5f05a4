# segment length sweep with paired head rows (TQR_SEGLEN; default 8)
set -o pipefail
OUT=gpurun_out/c31; mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
for S in 8 6 10 12 16; do
  TQR_SEGLEN=$S timeout -k 10 120 python bench.py --no-cpu-baseline --no-host-api --steps 10 --warmup 2 > $OUT/bench_s${S}_$r.json 2> $OUT/bench_s${S}_$r.err || { echo "bench $S failed"; tail -20 $OUT/bench_s${S}_$r.err; exit 1; }
  echo "seglen $S $(python3 -c "import json,sys; d=json.load(open('$OUT/bench_s${S}_$r.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'])")"
done
done
