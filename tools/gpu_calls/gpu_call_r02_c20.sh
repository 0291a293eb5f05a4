set -o pipefail
mkdir -p gpurun_out/r02_c20
for v in vhead vsoff; do
  TQR_LIB=libtqr_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-api --steps 5 --warmup 2 --storage f32 --rows 32768 --cols 32768 > gpurun_out/r02_c20/bench_$v.json 2> gpurun_out/r02_c20/bench_$v.err || { echo bench failed; tail gpurun_out/r02_c20/bench_$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r02_c20/bench_$v.json').read());print('$v', d['ms_per_step'], d['roofline']['frac'], d.get('status'))"
done
