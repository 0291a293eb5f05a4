set -o pipefail
mkdir -p gpurun_out/r02_c48
for lib in libtqr.so libtqr_pt64.so libtqr_pt256.so libtqr_pt128.so libtqr.so libtqr_pt64.so; do
  TQR_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-api --steps 5 > gpurun_out/r02_c48/d_$lib.json 2>/dev/null || { echo bench failed; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r02_c48/d_$lib.json').read());print('f64', '$lib', d['ms_per_step'])"
done
for lib in libtqr.so libtqr_pt64.so libtqr_pt256.so libtqr.so; do
  TQR_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-api --steps 3 --warmup 1 --storage f32 --rows 32768 --cols 32768 > gpurun_out/r02_c48/f_$lib.json 2>/dev/null || { echo bench failed; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r02_c48/f_$lib.json').read());print('f32', '$lib', d['ms_per_step'])"
done
TQR_LIB=libtqr_pt64.so timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "flow or engine or plan" > gpurun_out/r02_c48/pytest_pt64.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/r02_c48/pytest_pt64.log; exit 1; }
tail -2 gpurun_out/r02_c48/pytest_pt64.log
