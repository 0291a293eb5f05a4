set -o pipefail
mkdir -p gpurun_out/r02_c38
for v in libtqr.so libtqr_fine.so libtqr.so libtqr_fine.so; do
  TQR_LIB=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-api --steps 10 > gpurun_out/r02_c38/bench_$v.json 2> gpurun_out/r02_c38/bench_$v.err || { echo bench failed; tail gpurun_out/r02_c38/bench_$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r02_c38/bench_$v.json').read());print('$v', d['ms_per_step'], d['roofline']['frac'])"
done
