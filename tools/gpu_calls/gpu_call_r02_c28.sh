# bench with staged inputs: default run (as the driver), the restore fallback (--steps 50), 2-rank rehearsal
set -o pipefail
OUT=gpurun_out/c28; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench default failed"; tail -20 $OUT/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_default.json')); print('default', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['config']['inputs'], d['check'])"
timeout -k 10 300 python bench.py --steps 50 --warmup 2 --no-cpu-baseline --no-host-api > $OUT/bench_50.json 2> $OUT/bench_50.err || { echo "bench 50 failed"; tail -20 $OUT/bench_50.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_50.json')); print('steps50', d['ms_per_step'], d['value'], d['config']['inputs'], d['check'])"
TQR_BENCH_DEVICE=0 TQR_BENCH_BACKEND=gloo TQR_FLOW_GRID=128 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/reh.json 2> $OUT/reh.err || { echo "rehearsal failed"; tail -20 $OUT/reh.err; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/reh.json').read().strip().splitlines()[-1]);print('reh', d['ms_per_step'], d['value'], d['config']['inputs'], json.dumps(d['dist'])[:300])"
