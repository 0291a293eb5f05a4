# HEAD (panel-side forwarding) full GPU suite; panel trailing on apply_x4 (px4): parity subset, A/B x3, stamps
set -o pipefail
OUT=gpurun_out/c26; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -x -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu_head.log 2>&1 || { echo "pytest HEAD failed"; tail -30 $OUT/pytest_gpu_head.log; exit 1; }
tail -1 $OUT/pytest_gpu_head.log
TQR_LIB=libtqr_px4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_factor.py tests/test_gpu_tiles.py -q -x -m gpu --timeout 120 --timeout-method thread -k "vs_oracle or vs_reference or structured or fp32 or c3" > $OUT/pytest_px4.log 2>&1 || { echo "pytest px4 failed"; tail -30 $OUT/pytest_px4.log; exit 1; }
tail -1 $OUT/pytest_px4.log
for r in 1 2 3; do
for L in libtqr.so libtqr_px4.so; do
  TQR_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline --no-host-api --steps 10 --warmup 2 > $OUT/bench_${L}_$r.json 2> $OUT/bench_${L}_$r.err || { echo "bench $L failed"; tail -20 $OUT/bench_${L}_$r.err; exit 1; }
  echo "$L $(python3 -c "import json,sys; d=json.load(open('$OUT/bench_${L}_$r.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'])")"
done
done
for F in libtqr_fst.so libtqr_diag_px4.so; do
  TQR_FST_LIB=$F timeout -k 10 120 python tools/flowstamps.py 16384 > $OUT/fst_$F.txt 2>&1 || { echo "stamps $F failed"; tail -20 $OUT/fst_$F.txt; exit 1; }
  grep -E "wall|per panel group" $OUT/fst_$F.txt
done
