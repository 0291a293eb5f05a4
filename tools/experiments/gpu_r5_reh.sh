#!/bin/bash
# New parity cases (chain knobs, fp32 asm shapes, the 8-GPU defaults at 4 ranks), then the one-GPU
# rehearsals at 65536x16384 (2 ranks x 128 CUs, 4 ranks x 64 CUs at the rehearsal defaults, and 4
# ranks with the 8-GPU defaults forced), and the one-GPU c4 line.
set -o pipefail
O=gpurun_out/${1:-reh5}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_factor.py tests/test_dist.py -x -v --timeout 300 --timeout-method thread \
  -k "chain_knobs or test_factor_vs_oracle or ranks_on_one_gpu" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
R="TQR_BENCH_DEVICE=0 TQR_BENCH_BACKEND=gloo"
env TQR_BENCH_DEVICE=0 TQR_BENCH_BACKEND=gloo TQR_FLOW_GRID=128 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > $O/r2.json 2> $O/r2.err || { echo "2-rank failed"; tail -20 $O/r2.err; exit 1; }
tail -1 $O/r2.json | cut -c1-400
env TQR_BENCH_DEVICE=0 TQR_BENCH_BACKEND=gloo TQR_FLOW_GRID=64 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 4 --steps 3 --warmup 1 --no-cpu-baseline > $O/r4.json 2> $O/r4.err || { echo "4-rank failed"; tail -20 $O/r4.err; exit 1; }
tail -1 $O/r4.json | cut -c1-400
env TQR_BENCH_DEVICE=0 TQR_BENCH_BACKEND=gloo TQR_FLOW_GRID=64 TQR_SEGLEN=2 TQR_TAIL=28 TQR_TAIL_SEGLEN=1 TQR_LAC=4 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29543 bench.py --gpus 4 --steps 3 --warmup 1 --no-cpu-baseline > $O/r4_8gpu_defaults.json 2> $O/r4b.err || { echo "4-rank (8-GPU defaults) failed"; tail -20 $O/r4b.err; exit 1; }
tail -1 $O/r4_8gpu_defaults.json | cut -c1-400
timeout -k 10 300 python bench.py --rows 65536 --cols 16384 --no-cpu-baseline --no-host-api > $O/c4.json 2> $O/c4.err || { echo "c4 failed"; tail -20 $O/c4.err; exit 1; }
cut -c1-300 $O/c4.json
