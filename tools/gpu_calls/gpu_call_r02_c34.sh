# final HEAD (nt head loads): full GPU suite; element-start head loads nt as well (A/B x2); default bench; rocprof
set -o pipefail
OUT=gpurun_out/c34; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -x -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for r in 1 2; do
for L in libtqr.so libtqr_h0.so; do
  TQR_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline --no-host-api --steps 10 --warmup 2 > $OUT/bench_${L}_$r.json 2> $OUT/bench_${L}_$r.err || { echo "bench $L failed"; tail -20 $OUT/bench_${L}_$r.err; exit 1; }
  echo "$L $(python3 -c "import json,sys; d=json.load(open('$OUT/bench_${L}_$r.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'])")"
done
done
timeout -k 10 400 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench default failed"; tail -20 $OUT/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_default.json')); print('default', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['check'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-host-api --steps 2 --warmup 1 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
grep k_flow $OUT/prof/prof_kernel_stats.csv | cut -c1-200
