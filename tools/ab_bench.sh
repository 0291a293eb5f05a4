#!/bin/bash
# A/B timing of variants on the GPU box: bash tools/ab_bench.sh OUT ROUNDS VARIANT ...
# VARIANT = lib.so[:NAME=VALUE[,NAME=VALUE...]] — a library by file name in
# gpu-tiled-qr-decomposition_amd/ (loaded via TQR_LIB) and optional environment settings.
# Variants alternate round by round; BENCH_ARGS adds bench flags; the first failure ends the script.
set -o pipefail
O=$1; R=$2; shift 2
mkdir -p $O
for r in $(seq 1 $R); do
  for V in "$@"; do
    L=${V%%:*}; E=""; [ "$V" != "$L" ] && E=${V#*:}
    tag=$(echo "${L%.so}_${E}" | tr ',=' '__')
    env TQR_LIB=$L $(echo $E | tr ',' ' ') timeout -k 10 240 python bench.py --no-cpu-baseline --no-host-api ${BENCH_ARGS:-} > $O/${tag}_$r.json 2>> $O/ab.err || { echo "bench $V failed"; tail -5 $O/ab.err; exit 1; }
    python -c "import json;d=json.load(open('$O/${tag}_$r.json'));print('$V', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
  done
done
