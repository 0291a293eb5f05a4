set -o pipefail
mkdir -p gpurun_out/r02_c39
timeout -k 10 400 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -k "f32 or fp32 or float32" > gpurun_out/r02_c39/pytest_f32.log 2>&1 || { echo "pytest failed"; grep -E "^FAILED|passed|failed" gpurun_out/r02_c39/pytest_f32.log; exit 1; }
tail -1 gpurun_out/r02_c39/pytest_f32.log
timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-api --steps 5 --warmup 2 --storage f32 --rows 32768 --cols 32768 > gpurun_out/r02_c39/bench_f32.json 2> gpurun_out/r02_c39/bench_f32.err || { echo bench failed; tail gpurun_out/r02_c39/bench_f32.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r02_c39/bench_f32.json').read());print(d['ms_per_step'], d['roofline']['frac'])"
