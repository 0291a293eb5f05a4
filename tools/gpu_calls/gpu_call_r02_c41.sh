set -o pipefail
mkdir -p gpurun_out/r02_c41
TQR_FST_LIB=libtqr_fst.so TQR_TIMELINE_DUMP=gpurun_out/r02_c41/timeline.npz timeout -k 10 200 python tools/timeline.py 16384 > gpurun_out/r02_c41/timeline.txt 2>&1 || { echo timeline failed; tail gpurun_out/r02_c41/timeline.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r02_c41/timeline.txt
