set -o pipefail
mkdir -p gpurun_out/r02_c27
for v in fst diag_NOBARRIER diag_NODRAIN diag_NODMA diag_NOSTRIP diag_NOHEAD; do
  echo "== $v"
  TQR_FST_LIB=libtqr_$v.so timeout -k 10 100 python tools/flowstamps.py 16384 > gpurun_out/r02_c27/fst_$v.txt 2>&1 || { echo "fst $v failed"; tail -3 gpurun_out/r02_c27/fst_$v.txt; }
  grep -E "wall|phase|drain|barrier|head|strip" gpurun_out/r02_c27/fst_$v.txt
done
