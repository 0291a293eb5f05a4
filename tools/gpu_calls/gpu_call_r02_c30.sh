set -o pipefail
mkdir -p gpurun_out/r02_c30
TQR_FST_LIB=libtqr_fst.so timeout -k 10 200 python tools/flowstamps.py 16384 > gpurun_out/r02_c30/fst.txt 2>&1 || { echo "fst failed"; tail gpurun_out/r02_c30/fst.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r02_c30/fst.txt
