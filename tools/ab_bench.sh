#!/bin/bash
# A/B timing of library variants on the GPU box: bash tools/ab_bench.sh OUT ROUNDS lib_a.so lib_b.so ...
# (each lib by file name in gpu-tiled-qr-decomposition_amd/, loaded via TQR_LIB; BENCH_ARGS extra bench flags)
# Variants alternate round by round; one bench per (round, lib); the first failure ends the script.
set -o pipefail
O=$1; R=$2; shift 2
mkdir -p $O
for r in $(seq 1 $R); do
  for L in "$@"; do
    TQR_LIB=$L timeout -k 10 240 python bench.py --no-cpu-baseline --no-host-api ${BENCH_ARGS:-} > $O/${L%.so}_$r.json 2>> $O/ab.err || { echo "bench $L failed"; tail -5 $O/ab.err; exit 1; }
    python -c "import json;d=json.load(open('$O/${L%.so}_$r.json'));print('$L', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
  done
done
