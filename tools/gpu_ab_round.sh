#!/bin/bash
# One GPU-box pass for candidate libraries: a parity run on the candidate, then alternating A/B
# timing against the shipped library (and any other variants).
#   bash tools/gpu_ab_round.sh TAG CANDIDATE.so [ROUNDS]
# Environment (all optional):
#   TESTS=0            skip the parity run
#   PYTEST_FILES="..." test files of the parity run (default: the whole GPU suite, tests/)
#   PYTEST_K="..."     a -k selection for it
#   BASE=lib.so        the library the candidate is timed against (default libtqr.so)
#   EXTRA_VARIANTS="lib.so[:K=V,...] ..."  more variants in the alternation (tools/ab_bench.sh syntax)
#   BENCH_ARGS="..."   bench.py flags (e.g. --no-single-leg, --dtype f32 ...)
# Each GPU step has its own time limit; the first failure ends the script (no retries).
# (Round 6: this replaces the one-shot tools/experiments/gpu_r5_*.sh scripts, which were this pass
# with a fixed candidate, test selection and variant list.)
set -o pipefail
TAG=$1; CAND=$2; R=${3:-2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  K=(); [ -n "${PYTEST_K:-}" ] && K=(-k "$PYTEST_K")
  TQR_LIB=$CAND timeout -k 10 900 python -u -m pytest ${PYTEST_FILES:-tests} -q -x -m gpu --timeout 300 --timeout-method thread "${K[@]}" > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -n 2 $OUT/pytest_gpu.log
fi
bash tools/ab_bench.sh $OUT/ab $R ${BASE:-libtqr.so} $CAND ${EXTRA_VARIANTS:-}
