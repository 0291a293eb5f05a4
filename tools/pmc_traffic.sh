#!/bin/bash
# HBM-side traffic of one k_flow launch (16384^2, b=256): two rocprofv3 --pmc passes (one counter
# each, no trace domains), then tools/pmc_summary.py writes profiles/pmc_summary.json.
# Output CSVs under gpurun_out/pmc/<counter>/ (copy to profiles/ to keep them).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/pmc/$c -o pmc --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/pmc/$c.log 2>&1 || { echo "pmc $c failed"; tail -20 gpurun_out/pmc/$c.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc
