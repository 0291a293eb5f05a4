# A/B: fp64 chain at one wave per SIMD (TQR_NT64=256, 32 columns per wave) vs the shipped 8-wave form
set -o pipefail
OUT=gpurun_out/c20; mkdir -p $OUT
export TMPDIR=/tmp
TQR_LIB=libtqr_w32.so timeout -k 10 300 python -u -m pytest tests/test_gpu_factor.py -q -x -m gpu --timeout 120 --timeout-method thread -k "vs_oracle or vs_reference or structured" > $OUT/pytest_w32.log 2>&1 || { echo "pytest w32 failed"; tail -30 $OUT/pytest_w32.log; exit 1; }
tail -2 $OUT/pytest_w32.log
for r in 1 2; do
for L in libtqr.so libtqr_w32.so; do
  TQR_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline --no-host-api --steps 10 --warmup 2 > $OUT/bench_${L}_$r.json 2> $OUT/bench_${L}_$r.err || { echo "bench $L failed"; tail -20 $OUT/bench_${L}_$r.err; exit 1; }
  echo "$L $(python3 -c "import json,sys; d=json.load(open('$OUT/bench_${L}_$r.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'])")"
done
done
