set -o pipefail
mkdir -p gpurun_out/r02_c50
for lib in libtqr.so libtqr_c448.so libtqr_c448p384.so libtqr_c448p256.so libtqr_c320p256.so libtqr_c448.so libtqr_c448p384.so libtqr_c448p256.so; do
  TQR_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-api --steps 5 > gpurun_out/r02_c50/d_$lib.json 2>/dev/null || { echo bench failed; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r02_c50/d_$lib.json').read());print('f64', '$lib', d['ms_per_step'])"
done
