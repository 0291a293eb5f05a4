# Rc prefetch held one counter per lane of the poll wave (no scratch spill): parity subset, A/B x3 fp64, fp32 A/B
set -o pipefail
OUT=gpurun_out/c23; mkdir -p $OUT
export TMPDIR=/tmp
TQR_LIB=libtqr_pf.so timeout -k 10 300 python -u -m pytest tests/test_gpu_factor.py tests/test_gpu_tiles.py -q -x -m gpu --timeout 120 --timeout-method thread -k "vs_oracle or vs_reference or structured or fp32" > $OUT/pytest_pf.log 2>&1 || { echo "pytest pf failed"; tail -30 $OUT/pytest_pf.log; exit 1; }
tail -2 $OUT/pytest_pf.log
for r in 1 2 3; do
for L in libtqr.so libtqr_pf.so; do
  TQR_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline --no-host-api --steps 10 --warmup 2 > $OUT/bench_${L}_$r.json 2> $OUT/bench_${L}_$r.err || { echo "bench $L failed"; tail -20 $OUT/bench_${L}_$r.err; exit 1; }
  echo "$L $(python3 -c "import json,sys; d=json.load(open('$OUT/bench_${L}_$r.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'])")"
done
done
for L in libtqr.so libtqr_pf.so; do
  TQR_LIB=$L timeout -k 10 120 python bench.py --storage f32 --rows 32768 --cols 32768 --no-cpu-baseline --no-host-api --steps 4 --warmup 1 > $OUT/bench32_${L}.json 2> $OUT/bench32_${L}.err || { echo "bench32 $L failed"; tail -20 $OUT/bench32_${L}.err; exit 1; }
  echo "f32 $L $(python3 -c "import json,sys; d=json.load(open('$OUT/bench32_${L}.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'])")"
done
