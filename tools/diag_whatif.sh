#!/bin/bash
# What-if timings of the stamped engine (libtqr_diag_*.so, results wrong by construction):
# one flowstamps run per variant named in $VARIANTS. Output: gpurun_out/whatif/<variant>.txt
set -o pipefail
mkdir -p gpurun_out/whatif
for v in ${VARIANTS:-DMA_FIXED NODMA NOHEAD NOSTRIP}; do
  TQR_FST_LIB=libtqr_diag_$v.so timeout -k 10 120 python tools/flowstamps.py ${FST_ARGS:-16384} > gpurun_out/whatif/$v.txt 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/whatif/$v.txt; exit 1; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/whatif/$v.txt
done
