#!/bin/bash
# Round 6: per-wave stamps of the fp64 asm chain with slot 7 split (task start wait / task end /
# loop), plus the task timeline dump (tools/timeline.py). Diagnostic builds only.
set -o pipefail
O=gpurun_out/${1:-r6stamps}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/flowstamps.py 16384 > $O/flowstamps_f64.txt 2>&1 || exit 1
TQR_TIMELINE_DUMP=$O/timeline_f64.npz timeout -k 10 300 python -u tools/timeline.py 16384 > $O/timeline_f64.txt 2>&1 || exit 1
