set -o pipefail
mkdir -p gpurun_out/r02_c2
timeout -k 10 300 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread > gpurun_out/r02_c2/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r02_c2/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r02_c2/pytest_gpu.log
timeout -k 10 120 tools/ubench/mfma_f64 > gpurun_out/r02_c2/ubench_mfma.txt 2>&1 || { echo ubench failed; exit 1; }
cat gpurun_out/r02_c2/ubench_mfma.txt
VARIANTS="NOPTRAIL NOPFACT NOBT PANEL0" bash tools/diag_whatif.sh || exit 1
PMC_OUT=gpurun_out/r02_c2/pmc bash tools/pmc_traffic.sh || exit 1
