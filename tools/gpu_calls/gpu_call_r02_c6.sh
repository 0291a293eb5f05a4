set -o pipefail
mkdir -p gpurun_out/r02_c6
timeout -k 10 120 python tools/flowstamps.py 16384 > gpurun_out/r02_c6/fst.txt 2>&1 || { echo fst failed; tail gpurun_out/r02_c6/fst.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r02_c6/fst.txt
VARIANTS="NOHEAD NODMA NOSTRIP DMA_FIXED" bash tools/diag_whatif.sh || exit 1
