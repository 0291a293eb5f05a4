set -o pipefail
mkdir -p gpurun_out/r02_c37
timeout -k 10 400 python -u -m pytest tests -q -x -m gpu --timeout 300 --timeout-method thread -k "not 65536 and not 32768 and not f32" > gpurun_out/r02_c37/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "^FAILED|passed|failed" gpurun_out/r02_c37/pytest_gpu.log; tail -30 gpurun_out/r02_c37/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r02_c37/pytest_gpu.log
for v in libtqr.so libtqr_x2.so libtqr.so libtqr_x2.so; do
  TQR_LIB=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-api --steps 10 > gpurun_out/r02_c37/bench_$v.json 2> gpurun_out/r02_c37/bench_$v.err || { echo bench failed; tail gpurun_out/r02_c37/bench_$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r02_c37/bench_$v.json').read());print('$v', d['ms_per_step'], d['roofline']['frac'])"
done
TQR_FST_LIB=libtqr_fst.so timeout -k 10 200 python tools/flowstamps.py 16384 > gpurun_out/r02_c37/fst.txt 2>&1 || { echo "fst failed"; tail gpurun_out/r02_c37/fst.txt; exit 1; }
grep -E "wall|wave" gpurun_out/r02_c37/fst.txt
