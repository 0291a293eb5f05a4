set -o pipefail
mkdir -p gpurun_out/r02_c43
timeout -k 10 400 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -k "f32 or fp32 or float32" > gpurun_out/r02_c43/pytest_f32.log 2>&1 || { echo "pytest failed"; grep -E "^FAILED|passed|failed" gpurun_out/r02_c43/pytest_f32.log; exit 1; }
tail -1 gpurun_out/r02_c43/pytest_f32.log
for v in libtqr.so libtqr_p0.so libtqr.so libtqr_p0.so; do
  TQR_LIB=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-api --steps 3 --warmup 1 --storage f32 --rows 32768 --cols 32768 > gpurun_out/r02_c43/b_$v.json 2>/dev/null || { echo bench failed; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r02_c43/b_$v.json').read());print('$v', d['ms_per_step'])"
done
