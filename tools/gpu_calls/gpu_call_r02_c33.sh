set -o pipefail
mkdir -p gpurun_out/r02_c33
timeout -k 10 120 tools/ubench/mfma_f64 > gpurun_out/r02_c33/ubench_mfma.txt 2>&1
cat gpurun_out/r02_c33/ubench_mfma.txt | grep -E "4x4x4|device"
