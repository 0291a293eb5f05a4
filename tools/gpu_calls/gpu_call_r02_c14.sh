set -o pipefail
mkdir -p gpurun_out/r02_c14
timeout -k 10 60 tools/ubench/mfma_probe32 > gpurun_out/r02_c14/ubench_mfma_probe32.txt 2>&1 && tail -1 gpurun_out/r02_c14/ubench_mfma_probe32.txt
timeout -k 10 840 python -u -m pytest tests -q -x -m gpu --timeout 600 --timeout-method thread > gpurun_out/r02_c14/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" gpurun_out/r02_c14/pytest_gpu.log | head -30; tail -30 gpurun_out/r02_c14/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r02_c14/pytest_gpu.log
