# fp32 c5 and fp64 c3: nt strip loads (HEAD) vs sc1 strip loads, A/B x2 on one box
set -o pipefail
OUT=gpurun_out/c37; mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
for L in libtqr.so libtqr_sld16.so; do
  TQR_LIB=$L timeout -k 10 200 python bench.py --storage f32 --rows 32768 --cols 32768 --no-cpu-baseline --no-host-api --steps 4 --warmup 1 > $OUT/f32_${L}_$r.json 2> $OUT/f32_${L}_$r.err || { echo "bench f32 $L failed"; tail -20 $OUT/f32_${L}_$r.err; exit 1; }
  echo "f32 $L $(python3 -c "import json,sys; d=json.load(open('$OUT/f32_${L}_$r.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'])")"
  TQR_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline --no-host-api --steps 10 --warmup 2 > $OUT/f64_${L}_$r.json 2> $OUT/f64_${L}_$r.err || { echo "bench f64 $L failed"; tail -20 $OUT/f64_${L}_$r.err; exit 1; }
  echo "f64 $L $(python3 -c "import json,sys; d=json.load(open('$OUT/f64_${L}_$r.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'])")"
done
done
