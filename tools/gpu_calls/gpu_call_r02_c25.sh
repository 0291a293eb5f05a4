# panel-side forwarding (TQR_PANEL_FWD, no FWD tasks): dist parity on one GPU, rehearsal A/B (2 ranks x 128 CUs), stamps
set -o pipefail
OUT=gpurun_out/c25; mkdir -p $OUT
export TMPDIR=/tmp
TQR_LIB=libtqr_pfwd.so timeout -k 10 600 python -u -m pytest tests/test_dist.py -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_dist_pfwd.log 2>&1 || { echo "pytest dist pfwd failed"; tail -30 $OUT/pytest_dist_pfwd.log; exit 1; }
tail -2 $OUT/pytest_dist_pfwd.log
n=0
for r in 1 2; do
for L in libtqr.so libtqr_pfwd.so; do
n=$((n+1))
TQR_LIB=$L TQR_BENCH_DEVICE=0 TQR_BENCH_BACKEND=gloo TQR_FLOW_GRID=128 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2954$n bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/reh_${L}_$r.json 2> $OUT/reh_${L}_$r.err || { echo "rehearsal $L failed"; tail -20 $OUT/reh_${L}_$r.err; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/reh_${L}_$r.json').read().strip().splitlines()[-1]);print('$L', d['ms_per_step'], d['value'], [x['column_norm_rel_err'] for x in d['dist']['ranks']])"
done
done
for L in libtqr_fst.so libtqr_diag_pfwd.so; do
TQR_LIB=$L TQR_BENCH_DEVICE=0 TQR_BENCH_BACKEND=gloo TQR_FLOW_GRID=128 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29549 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/reh_stamps_$L.json 2> $OUT/reh_stamps_$L.err || { echo "stamps $L failed"; tail -20 $OUT/reh_stamps_$L.err; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/reh_stamps_$L.json').read().strip().splitlines()[-1]);print('$L', d['ms_per_step'], json.dumps(d['dist'])[:500])"
done
