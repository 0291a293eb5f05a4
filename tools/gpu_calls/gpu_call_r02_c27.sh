# fp64 chain poll thread on a lower wave (1, 2, 3) vs wave 7 (HEAD): A/B x3
set -o pipefail
OUT=gpurun_out/c27; mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2 3; do
for L in libtqr.so libtqr_pt64.so libtqr_pt128.so libtqr_pt192.so; do
  TQR_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline --no-host-api --steps 10 --warmup 2 > $OUT/bench_${L}_$r.json 2> $OUT/bench_${L}_$r.err || { echo "bench $L failed"; tail -20 $OUT/bench_${L}_$r.err; exit 1; }
  echo "$L $(python3 -c "import json,sys; d=json.load(open('$OUT/bench_${L}_$r.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'])")"
done
done
