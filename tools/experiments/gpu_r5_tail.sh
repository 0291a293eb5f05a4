#!/bin/bash
# fp64 16384^2 tail: task timeline of the last 8 steps (stamps build), then the PMC passes of the
# current library (executed flops after the UNMQR skip).
set -o pipefail
O=gpurun_out/${1:-tail}
mkdir -p $O
export TMPDIR=/tmp
TQR_TIMELINE_TAIL=8 timeout -k 10 300 python tools/timeline.py 16384 256 > $O/timeline_f64.txt 2>&1 || { echo "timeline failed"; tail -20 $O/timeline_f64.txt; exit 1; }
head -30 $O/timeline_f64.txt
PMC_OUT=$O/pmc bash tools/pmc_traffic.sh
