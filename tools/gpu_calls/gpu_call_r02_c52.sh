set -o pipefail
mkdir -p gpurun_out/r02_c52
timeout -k 10 900 python -u -m pytest tests -q -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/r02_c52/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" gpurun_out/r02_c52/pytest_gpu.log | head -20; tail -30 gpurun_out/r02_c52/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r02_c52/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r02_c52/bench.json 2> gpurun_out/r02_c52/bench.err || { echo bench failed; tail gpurun_out/r02_c52/bench.err; exit 1; }
cat gpurun_out/r02_c52/bench.json
timeout -k 10 120 python tools/flowstamps.py 16384 > gpurun_out/r02_c52/fst.txt 2>&1 || { echo fst failed; tail gpurun_out/r02_c52/fst.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r02_c52/fst.txt | tail -30
