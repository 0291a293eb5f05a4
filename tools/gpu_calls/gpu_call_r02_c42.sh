set -o pipefail
mkdir -p gpurun_out/r02_c42
for sl in 8 4 6 12 16 8; do
  TQR_SEGLEN=$sl timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-api --steps 5 > gpurun_out/r02_c42/b_$sl.json 2>/dev/null || { echo bench failed; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r02_c42/b_$sl.json').read());print('f64 seglen $sl', d['ms_per_step'])"
done
for sl in 8 16 4; do
  TQR_SEGLEN=$sl timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-api --steps 3 --warmup 1 --storage f32 --rows 32768 --cols 32768 > gpurun_out/r02_c42/f_$sl.json 2>/dev/null || { echo bench failed; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r02_c42/f_$sl.json').read());print('f32 seglen $sl', d['ms_per_step'])"
done
