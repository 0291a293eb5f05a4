# final HEAD: 2-rank rehearsal (2 x 128 CUs, 65536x16384) and c4 on one GPU
set -o pipefail
OUT=gpurun_out/c32; mkdir -p $OUT
export TMPDIR=/tmp
TQR_BENCH_DEVICE=0 TQR_BENCH_BACKEND=gloo TQR_FLOW_GRID=128 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/reh.json 2> $OUT/reh.err || { echo "rehearsal failed"; tail -20 $OUT/reh.err; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/reh.json').read().strip().splitlines()[-1]);print('reh', d['ms_per_step'], d['value'], json.dumps(d['dist'])[:300])"
timeout -k 10 300 python bench.py --rows 65536 --cols 16384 --steps 5 --warmup 1 --no-cpu-baseline --no-host-api > $OUT/c4_1gpu.json 2> $OUT/c4_1gpu.err || { echo "c4 failed"; tail -20 $OUT/c4_1gpu.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/c4_1gpu.json')); print('c4 1gpu', d['ms_per_step'], d['value'], d['roofline']['frac'], d['check'])"
