# c4 (65536x16384) on one GPU (t(1 GPU) of the strong-scaling ratio) and one rank on 128 CUs, staged inputs
set -o pipefail
OUT=gpurun_out/c29; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --rows 65536 --cols 16384 --steps 5 --warmup 1 --no-cpu-baseline --no-host-api > $OUT/c4_1gpu.json 2> $OUT/c4_1gpu.err || { echo "c4 failed"; tail -20 $OUT/c4_1gpu.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/c4_1gpu.json')); print('c4 1gpu', d['ms_per_step'], d['value'], d['roofline']['frac'], d['check'])"
TQR_FLOW_GRID=128 timeout -k 10 300 python bench.py --rows 65536 --cols 16384 --steps 3 --warmup 1 --no-cpu-baseline --no-host-api > $OUT/c4_128cu.json 2> $OUT/c4_128cu.err || { echo "c4 128cu failed"; tail -20 $OUT/c4_128cu.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/c4_128cu.json')); print('c4 128 CUs', d['ms_per_step'], d['value'], d['check'])"
