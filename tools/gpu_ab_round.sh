#!/bin/bash
# One GPU-box pass for a candidate library: parity suite on it, then alternating A/B timing against
# the shipped library. Usage: bash tools/gpu_ab_round.sh TAG CANDIDATE.so [ROUNDS]
# Each GPU step has its own time limit; the first failure ends the script (no retries).
set -o pipefail
TAG=$1; CAND=$2; R=${3:-2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  TQR_LIB=$CAND timeout -k 10 900 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
bash tools/ab_bench.sh $OUT/ab $R libtqr.so $CAND ${EXTRA_VARIANTS:-}
