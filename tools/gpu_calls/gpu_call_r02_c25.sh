set -o pipefail
mkdir -p gpurun_out/r02_c25
TQR_LIB=libtqr_v5.so timeout -k 10 200 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -k "factor_f32_b32 or factor_f32_b16" > gpurun_out/r02_c25/pytest_v5.log 2>&1; echo "v5 rc=$?"; tail -1 gpurun_out/r02_c25/pytest_v5.log
timeout -k 10 400 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -k "f32 or fp32 or float32" > gpurun_out/r02_c25/pytest_f32.log 2>&1 || { echo "pytest failed"; grep -E "^FAILED|passed|failed" gpurun_out/r02_c25/pytest_f32.log; exit 1; }
tail -1 gpurun_out/r02_c25/pytest_f32.log
timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-api --steps 5 --warmup 2 --storage f32 --rows 32768 --cols 32768 > gpurun_out/r02_c25/bench_f32.json 2> gpurun_out/r02_c25/bench_f32.err || { echo bench failed; tail gpurun_out/r02_c25/bench_f32.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r02_c25/bench_f32.json').read());print(d['ms_per_step'], d['roofline']['frac'])"
TQR_FST_LIB=libtqr_fst.so TQR_FST_DTYPE=f32 timeout -k 10 200 python tools/flowstamps.py 32768 > gpurun_out/r02_c25/fst.txt 2>&1 || { echo "fst failed"; tail gpurun_out/r02_c25/fst.txt; exit 1; }
grep -E "wall|phase|store|Rc wait in-elem other|strip|drain" gpurun_out/r02_c25/fst.txt
