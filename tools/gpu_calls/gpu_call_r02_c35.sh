# chain strip cache policy at HEAD: loads sc1|nt, stores sc1|nt, both; A/B x2 (parity subset on "both")
set -o pipefail
OUT=gpurun_out/c35; mkdir -p $OUT
export TMPDIR=/tmp
TQR_LIB=libtqr_sboth.so timeout -k 10 300 python -u -m pytest tests/test_gpu_factor.py -q -x -m gpu --timeout 120 --timeout-method thread -k "vs_oracle or vs_reference" > $OUT/pytest_sboth.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_sboth.log; exit 1; }
tail -1 $OUT/pytest_sboth.log
for r in 1 2; do
for L in libtqr.so libtqr_sld.so libtqr_sst.so libtqr_sboth.so; do
  TQR_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline --no-host-api --steps 10 --warmup 2 > $OUT/bench_${L}_$r.json 2> $OUT/bench_${L}_$r.err || { echo "bench $L failed"; tail -20 $OUT/bench_${L}_$r.err; exit 1; }
  echo "$L $(python3 -c "import json,sys; d=json.load(open('$OUT/bench_${L}_$r.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'])")"
done
done
