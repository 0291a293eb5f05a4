set -o pipefail
mkdir -p gpurun_out/r02_c22
timeout -k 10 400 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -k "f32 or fp32 or float32" > gpurun_out/r02_c22/pytest_f32.log 2>&1 || { echo "pytest failed"; grep -E "^FAILED|passed|failed" gpurun_out/r02_c22/pytest_f32.log; exit 1; }
tail -1 gpurun_out/r02_c22/pytest_f32.log
