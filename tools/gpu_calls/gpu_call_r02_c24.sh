# multi-GPU plans with uncached workspaces: dist parity tests (ranks on one GPU bit-exact vs one GPU),
# 2-rank rehearsal with the new per-rank output check, A/B against cached workspaces
set -o pipefail
OUT=gpurun_out/c24; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_dist.py -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_dist.log 2>&1 || { echo "pytest dist failed"; tail -30 $OUT/pytest_dist.log; exit 1; }
tail -3 $OUT/pytest_dist.log
for C in 0 1; do
TQR_DIST_WK_CACHED=$C TQR_BENCH_DEVICE=0 TQR_BENCH_BACKEND=gloo TQR_FLOW_GRID=128 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2953$C bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/two_ranks_cached$C.json 2> $OUT/two_ranks_cached$C.err || { echo "two-rank failed"; tail -20 $OUT/two_ranks_cached$C.err; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/two_ranks_cached$C.json').read().strip().splitlines()[-1]);print('cached=$C', d['ms_per_step'], d['value'], json.dumps(d['dist'])[:400])"
done
