set -o pipefail
mkdir -p gpurun_out/r02_c4
timeout -k 10 120 python tools/flowstamps.py 16384 > gpurun_out/r02_c4/fst.txt 2>&1 || { echo fst failed; tail gpurun_out/r02_c4/fst.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r02_c4/fst.txt
TQR_FST_LIB=libtqr_diag_PANEL0.so timeout -k 10 120 python tools/flowstamps.py 16384 > gpurun_out/r02_c4/fst_panel0.txt 2>&1 || { echo fst failed; exit 1; }
echo "== PANEL0"; grep -v amdgpu.ids gpurun_out/r02_c4/fst_panel0.txt
TQR_FST_LIB=libtqr_diag_PANEL0.so timeout -k 10 120 python tools/timeline.py 16384 > gpurun_out/r02_c4/timeline_panel0.txt 2>&1 || { echo tl failed; exit 1; }
echo "== PANEL0 timeline"; grep -v amdgpu.ids gpurun_out/r02_c4/timeline_panel0.txt | head -30
