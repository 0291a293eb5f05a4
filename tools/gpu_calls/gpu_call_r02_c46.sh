set -o pipefail
mkdir -p gpurun_out/r02_c46
TQR_FST_DTYPE=f32 TQR_FST_LIB=libtqr_fst.so timeout -k 10 200 python tools/timeline.py 32768 > gpurun_out/r02_c46/timeline_f32.txt 2>&1 || { echo timeline failed; tail gpurun_out/r02_c46/timeline_f32.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r02_c46/timeline_f32.txt
