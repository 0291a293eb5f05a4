# Multi-rank rehearsal on ONE GPU (2 ranks x 128 CUs over gloo): the bench's N=2 path at 65536x16384,
# against one rank on 128 CUs; then the same 2-rank run with the activity-stamps build to measure
# the CU time the forward tasks take (bench "dist" object: fwd_share_of_wg_time per rank).
set -o pipefail
mkdir -p gpurun_out/reh
TQR_BENCH_DEVICE=0 TQR_BENCH_BACKEND=gloo TQR_FLOW_GRID=128 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/reh/two_ranks.json 2> gpurun_out/reh/two_ranks.err || { echo "two-rank failed"; tail -20 gpurun_out/reh/two_ranks.err; exit 1; }
tail -1 gpurun_out/reh/two_ranks.json | cut -c1-300
TQR_FLOW_GRID=128 timeout -k 10 240 python bench.py --rows 65536 --cols 16384 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/reh/one_rank_128cu.json 2> gpurun_out/reh/one_rank.err || { echo "one-rank failed"; tail -20 gpurun_out/reh/one_rank.err; exit 1; }
tail -1 gpurun_out/reh/one_rank_128cu.json | cut -c1-300
TQR_LIB=libtqr_fst.so TQR_BENCH_DEVICE=0 TQR_BENCH_BACKEND=gloo TQR_FLOW_GRID=128 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/reh/two_ranks_stamps.json 2> gpurun_out/reh/two_ranks_stamps.err || { echo "two-rank stamps failed"; tail -20 gpurun_out/reh/two_ranks_stamps.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/reh/two_ranks_stamps.json').read().strip().splitlines()[-1]);print(json.dumps(d['dist']))"
