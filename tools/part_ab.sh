# A/B of the multi-GPU tile-column partition (snake, the default, vs TQR_DIST_PART=cyclic) in the
# one-GPU rehearsal at 65536x16384: 2 ranks x 128 CUs and 4 ranks x 64 CUs, alternating, with one
# rank on the same CU count as the reference point. Lines: part, ranks, ms per step, column check.
set -o pipefail
mkdir -p gpurun_out/part
run() {  # $1 part, $2 ranks, $3 CUs per rank, $4 tag
  TQR_DIST_PART=$1 TQR_BENCH_DEVICE=0 TQR_BENCH_BACKEND=gloo TQR_FLOW_GRID=$3 timeout -k 10 300 \
    python -m torch.distributed.run --nnodes=1 --nproc-per-node $2 --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 300)) \
    bench.py --gpus $2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/part/$4.json 2> gpurun_out/part/$4.err \
    || { echo "$4 failed"; tail -20 gpurun_out/part/$4.err; return 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/part/$4.json').read().strip().splitlines()[-1]);s=d['strong_scaling'];print('$1', $2, 'ranks x', $3, 'CUs:', d['ms_per_step'], 'ms; t1', s['t1_ms'], 'speedup', s['speedup'], [r['status'] for r in d['dist']['ranks']], max(r['column_norm_rel_err'] for r in d['dist']['ranks']))"
}
run snake 2 128 snake2a && run cyclic 2 128 cyclic2a && run snake 2 128 snake2b && run cyclic 2 128 cyclic2b &&
run snake 4 64 snake4a && run cyclic 4 64 cyclic4a && run snake 4 64 snake4b && run cyclic 4 64 cyclic4b
