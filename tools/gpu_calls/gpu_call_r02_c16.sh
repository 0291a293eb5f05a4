set -o pipefail
mkdir -p gpurun_out/r02_c16
timeout -k 10 840 python -u -m pytest tests -q -x -m gpu --timeout 600 --timeout-method thread > gpurun_out/r02_c16/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" gpurun_out/r02_c16/pytest_gpu.log | head -30; tail -30 gpurun_out/r02_c16/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r02_c16/pytest_gpu.log
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r02_c16/bench.json 2> gpurun_out/r02_c16/bench.err || { echo bench failed; tail gpurun_out/r02_c16/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r02_c16/bench.json').read());print(d['ms_per_step'], d['roofline']['frac'], json.dumps(d['host_api']))"
