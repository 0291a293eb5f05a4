# 16-B paired head rows in the fp64 chain (TQR_HEAD_PAIR): parity subset (incl. c3 elementwise), A/B x3, stamps
set -o pipefail
OUT=gpurun_out/c30; mkdir -p $OUT
export TMPDIR=/tmp
TQR_LIB=libtqr_hpair.so timeout -k 10 400 python -u -m pytest tests/test_gpu_factor.py tests/test_gpu_tiles.py tests/test_dist.py -q -x -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_hpair.log 2>&1 || { echo "pytest hpair failed"; tail -30 $OUT/pytest_hpair.log; exit 1; }
tail -1 $OUT/pytest_hpair.log
for r in 1 2 3; do
for L in libtqr.so libtqr_hpair.so; do
  TQR_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline --no-host-api --steps 10 --warmup 2 > $OUT/bench_${L}_$r.json 2> $OUT/bench_${L}_$r.err || { echo "bench $L failed"; tail -20 $OUT/bench_${L}_$r.err; exit 1; }
  echo "$L $(python3 -c "import json,sys; d=json.load(open('$OUT/bench_${L}_$r.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'])")"
done
done
TQR_FST_LIB=libtqr_diag_hpair.so timeout -k 10 120 python tools/flowstamps.py 16384 > $OUT/fst_hpair.txt 2>&1 || { echo "stamps failed"; tail -20 $OUT/fst_hpair.txt; exit 1; }
grep -A9 "per-wave" $OUT/fst_hpair.txt
