set -o pipefail
mkdir -p gpurun_out/r02_c54
for lib in libtqr_head.so libtqr.so libtqr_pvw.so libtqr_head.so libtqr.so libtqr_pvw.so; do
  TQR_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-api --steps 5 > gpurun_out/r02_c54/d_$lib.json 2>/dev/null || { echo bench failed; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r02_c54/d_$lib.json').read());print('f64', '$lib', d['ms_per_step'])"
done
for lib in libtqr_head.so libtqr.so libtqr_head.so libtqr.so; do
  TQR_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-api --steps 3 --warmup 1 --storage f32 --rows 32768 --cols 32768 > gpurun_out/r02_c54/f_$lib.json 2>/dev/null || { echo bench failed; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r02_c54/f_$lib.json').read());print('f32', '$lib', d['ms_per_step'])"
done
