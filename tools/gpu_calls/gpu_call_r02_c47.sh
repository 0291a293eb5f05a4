set -o pipefail
mkdir -p gpurun_out/r02_c47
for tg in 1.4 2.0 2.8 4.0 1.4; do
  TQR_TG=$tg timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-api --steps 3 --warmup 1 --storage f32 --rows 32768 --cols 32768 > gpurun_out/r02_c47/f_$tg.json 2>/dev/null || { echo bench failed; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r02_c47/f_$tg.json').read());print('f32 TG $tg', d['ms_per_step'])"
done
for tg in 1.0 2.0; do
  TQR_TG=$tg timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-api --steps 5 > gpurun_out/r02_c47/d_$tg.json 2>/dev/null || { echo bench failed; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r02_c47/d_$tg.json').read());print('f64 TG $tg', d['ms_per_step'])"
done
