set -o pipefail
mkdir -p gpurun_out/r02_c3
SEGS=8 SEGLAS=1,2,4,8 TGS=1.4 LAZYS=1 timeout -k 10 300 python tools/sweep_plan.py 16384 > gpurun_out/r02_c3/sweep.txt 2>&1 || { echo sweep failed; tail -5 gpurun_out/r02_c3/sweep.txt; exit 1; }
cat gpurun_out/r02_c3/sweep.txt
for la in 1 8; do
  TQR_SEGLEN_LA=$la TQR_FST_LIB=libtqr_diag_PANEL0.so timeout -k 10 120 python tools/flowstamps.py 16384 > gpurun_out/r02_c3/panel0_la$la.txt 2>&1 || { echo fst failed; exit 1; }
  echo "== PANEL0 la $la"; grep -v amdgpu.ids gpurun_out/r02_c3/panel0_la$la.txt | head -12
done
TQR_SEGLEN_LA=1 timeout -k 10 120 python tools/flowstamps.py 16384 > gpurun_out/r02_c3/fst_la1.txt 2>&1 || { echo fst failed; exit 1; }
echo "== base la 1"; grep -v amdgpu.ids gpurun_out/r02_c3/fst_la1.txt
