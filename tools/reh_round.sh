#!/bin/bash
# One GPU box, BASELINE configs[3] (65536 x 16384 fp64): the one-GPU run and the multi-rank
# rehearsals on that one GPU (N ranks over gloo, CUs / N workgroups each, the bench's own launcher),
# with the dist parity tests first. The numbers the 8-GPU model is calibrated against
# (tools/sched_sim.py calib).
#   bash tools/reh_round.sh TAG
# Each GPU step has its own time limit; the first failure ends the script (no retries).
set -o pipefail
TAG=${1:-reh}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_dist.py -q -x -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "dist tests failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --rows 65536 --cols 16384 --steps 3 --warmup 1 --no-cpu-baseline --no-host-api > $OUT/c4.json 2> $OUT/c4.err || { echo "c4 failed"; tail -20 $OUT/c4.err; exit 1; }
tail -n 1 $OUT/c4.json | cut -c1-200
for N in 2 4; do
  TQR_BENCH_DEVICE=0 TQR_BENCH_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus $N --steps 3 --warmup 1 --no-cpu-baseline > $OUT/r$N.json 2> $OUT/r$N.err || { echo "rehearsal $N failed"; tail -20 $OUT/r$N.err; exit 1; }
  tail -n 1 $OUT/r$N.json | cut -c1-200
done
# the 8-GPU task list (the whole-device multi-rank defaults) forced on the 4-rank rehearsal
TQR_SEGLEN=2 TQR_TAIL=28 TQR_TAIL_SEGLEN=1 TQR_LAC=4 TQR_BENCH_DEVICE=0 TQR_BENCH_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 4 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/r4_8gpu_defaults.json 2> $OUT/r4_8gpu_defaults.err || { echo "rehearsal 4 (8-GPU list) failed"; tail -20 $OUT/r4_8gpu_defaults.err; exit 1; }
tail -n 1 $OUT/r4_8gpu_defaults.json | cut -c1-200
