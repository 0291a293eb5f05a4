set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02_c40
mkdir -p $O
timeout -k 10 840 python -u -m pytest tests -q -x -m gpu --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "^FAILED|passed|failed" $O/pytest_gpu.log; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo bench failed; tail $O/bench_default.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench_default.json').read());print('default', d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_f64 -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-host-api --steps 5 --warmup 2 > $O/prof_f64.log 2>&1 || { echo rocprof failed; tail $O/prof_f64.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_f32 -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-host-api --steps 2 --warmup 1 --storage f32 --rows 32768 --cols 32768 > $O/prof_f32.log 2>&1 || { echo rocprof f32 failed; tail $O/prof_f32.log; exit 1; }
find $O/prof_f64 $O/prof_f32 -name "*kernel_stats.csv" -exec grep -H k_flow {} \; | cut -c1-220
PMC_OUT=$O/pmc BENCH_ARGS="--no-host-api" bash tools/pmc_traffic.sh || exit 1
PMC_OUT=$O/pmc_f32 PMC_KEY=32768x32768_b256_f32 BENCH_ARGS="--no-host-api --storage f32 --rows 32768 --cols 32768" bash tools/pmc_traffic.sh || exit 1
cp profiles/pmc_summary.json $O/pmc_summary.json
python3 -c "import json;d=json.load(open('$O/pmc_summary.json'));[print(k, round(v['update_hbm_bytes_per_launch']/1e9,1), 'GB util', round(v['mfma_util'],3)) for k,v in d.items() if not k.startswith('_')]"
