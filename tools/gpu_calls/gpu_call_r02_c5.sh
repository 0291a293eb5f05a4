set -o pipefail
mkdir -p gpurun_out/r02_c5
timeout -k 10 840 python -u -m pytest tests -v -x -m gpu --timeout 600 --timeout-method thread -s > gpurun_out/r02_c5/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/r02_c5/pytest_gpu.log | tail -40; tail -30 gpurun_out/r02_c5/pytest_gpu.log; exit 1; }
grep -E "passed|failed|c3 " gpurun_out/r02_c5/pytest_gpu.log | tail -5
timeout -k 10 120 python tools/flowstamps.py 16384 > gpurun_out/r02_c5/fst.txt 2>&1 || { echo fst failed; tail gpurun_out/r02_c5/fst.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r02_c5/fst.txt
