# final HEAD (nt strip + head loads): full GPU suite, default bench, rocprof kernel stats, fp32 c5 bench
set -o pipefail
OUT=${OUT:-gpurun_out/c36}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -x -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 400 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench default failed"; tail -20 $OUT/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_default.json')); print('default', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['check'])"
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-api > $OUT/bench_10.json 2> $OUT/bench_10.err || { echo "bench 10 failed"; tail -20 $OUT/bench_10.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_10.json')); print('steps10', d['ms_per_step'], d['value'], d['roofline']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-host-api --steps 2 --warmup 1 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
grep k_flow $OUT/prof/prof_kernel_stats.csv | cut -c1-200
timeout -k 10 300 python bench.py --storage f32 --rows 32768 --cols 32768 --no-cpu-baseline --no-host-api --steps 4 --warmup 1 > $OUT/bench_f32.json 2> $OUT/bench_f32.err || { echo "bench f32 failed"; tail -20 $OUT/bench_f32.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_f32.json')); print('f32 c5', d['ms_per_step'], d['value'], d['roofline']['frac'], d['check'])"
