#!/bin/bash
# fp32 c5 per-wave activity sums of the asm chain (stamps build): who waits at the group barrier.
set -o pipefail
O=gpurun_out/${1:-f32waves}
mkdir -p $O
export TMPDIR=/tmp
TQR_FST_DTYPE=f32 timeout -k 10 300 python tools/flowstamps.py 32768 32768 256 > $O/flowstamps_f32.txt 2>&1 || { echo "flowstamps failed"; tail -20 $O/flowstamps_f32.txt; exit 1; }
cat $O/flowstamps_f32.txt
timeout -k 10 300 python tools/flowstamps.py 16384 16384 256 > $O/flowstamps_f64.txt 2>&1 || { echo "flowstamps f64 failed"; tail -20 $O/flowstamps_f64.txt; exit 1; }
cat $O/flowstamps_f64.txt
