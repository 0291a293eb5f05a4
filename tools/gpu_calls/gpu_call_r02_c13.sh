set -o pipefail
mkdir -p gpurun_out/r02_c13
timeout -k 10 60 tools/ubench/mfma_probe32 > gpurun_out/r02_c13/ubench_mfma_probe32.txt 2>&1 || true
mkdir -p gpurun_out/r02_c13
timeout -k 10 600 python -u -m pytest tests -v -x -m gpu --timeout 300 --timeout-method thread -k "f32 or fp32 or float32" > gpurun_out/r02_c13/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" gpurun_out/r02_c13/pytest_gpu.log | head -30; tail -40 gpurun_out/r02_c13/pytest_gpu.log; exit 1; }
grep -E "PASS|passed|failed" gpurun_out/r02_c13/pytest_gpu.log | tail -30
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --storage f32 --rows 32768 --cols 32768 > gpurun_out/r02_c13/bench_f32.json 2> gpurun_out/r02_c13/bench_f32.err || { echo bench failed; tail gpurun_out/r02_c13/bench_f32.err; exit 1; }
cat gpurun_out/r02_c13/bench_f32.json
