# head-row I/O inside phase 2 (TQR_HEAD_IN_P2): parity subset, A/B bench x2, stamps
set -o pipefail
OUT=gpurun_out/c22; mkdir -p $OUT
export TMPDIR=/tmp
TQR_LIB=libtqr_hp2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_factor.py -q -x -m gpu --timeout 120 --timeout-method thread -k "vs_oracle or vs_reference or structured" > $OUT/pytest_hp2.log 2>&1 || { echo "pytest hp2 failed"; tail -30 $OUT/pytest_hp2.log; exit 1; }
tail -2 $OUT/pytest_hp2.log
for r in 1 2; do
for L in libtqr.so libtqr_hp2.so; do
  TQR_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline --no-host-api --steps 10 --warmup 2 > $OUT/bench_${L}_$r.json 2> $OUT/bench_${L}_$r.err || { echo "bench $L failed"; tail -20 $OUT/bench_${L}_$r.err; exit 1; }
  echo "$L $(python3 -c "import json,sys; d=json.load(open('$OUT/bench_${L}_$r.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'])")"
done
done
TQR_FST_LIB=libtqr_diag_hp2.so timeout -k 10 120 python tools/flowstamps.py 16384 > $OUT/fst_hp2.txt 2>&1 || { echo "stamps failed"; tail -20 $OUT/fst_hp2.txt; exit 1; }
