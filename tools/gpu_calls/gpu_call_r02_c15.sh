set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02_c15
timeout -k 10 400 python bench.py > gpurun_out/r02_c15/bench_default.json 2> gpurun_out/r02_c15/bench_default.err || { echo bench failed; tail gpurun_out/r02_c15/bench_default.err; exit 1; }
cat gpurun_out/r02_c15/bench_default.json
PMC_OUT=gpurun_out/r02_c15/pmc_f32 PMC_KEY=32768x32768_b256_f32 BENCH_ARGS="--storage f32 --rows 32768 --cols 32768" bash tools/pmc_traffic.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02_c15/prof_f32 -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --storage f32 --rows 32768 --cols 32768 > gpurun_out/r02_c15/prof_f32.log 2>&1 || { echo rocprof failed; tail gpurun_out/r02_c15/prof_f32.log; exit 1; }
find gpurun_out/r02_c15/prof_f32 -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-160
