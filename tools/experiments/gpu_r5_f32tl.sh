#!/bin/bash
# fp32 c5 after the asm chain: task timeline (occupancy per 5 %, the last steps) and the activity
# stamps (per-category and per-wave sums), stamps build.
set -o pipefail
O=gpurun_out/${1:-f32tl}
mkdir -p $O
export TMPDIR=/tmp
TQR_FST_DTYPE=f32 TQR_TIMELINE_TAIL=4 timeout -k 10 300 python tools/timeline.py 32768 256 > $O/timeline_f32.txt 2>&1 || { echo "timeline failed"; tail -20 $O/timeline_f32.txt; exit 1; }
head -28 $O/timeline_f32.txt
TQR_FST_DTYPE=f32 timeout -k 10 300 python tools/flowstamps.py 32768 32768 256 > $O/flowstamps_f32.txt 2>&1 || { echo "flowstamps failed"; tail -20 $O/flowstamps_f32.txt; exit 1; }
cat $O/flowstamps_f32.txt
