set -o pipefail
mkdir -p gpurun_out/r02_c26
timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-api > gpurun_out/r02_c26/bench.json 2> gpurun_out/r02_c26/bench.err || { echo bench failed; tail gpurun_out/r02_c26/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r02_c26/bench.json').read());print('f64', d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-api --steps 5 --warmup 2 --storage f32 --rows 32768 --cols 32768 > gpurun_out/r02_c26/bench_f32.json 2> gpurun_out/r02_c26/bench_f32.err || { echo bench failed; tail gpurun_out/r02_c26/bench_f32.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r02_c26/bench_f32.json').read());print('f32', d['ms_per_step'], d['roofline']['frac'])"
TQR_FST_LIB=libtqr_fst.so timeout -k 10 200 python tools/flowstamps.py 16384 > gpurun_out/r02_c26/fst.txt 2>&1 || { echo "fst failed"; tail gpurun_out/r02_c26/fst.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r02_c26/fst.txt | head -40
timeout -k 10 840 python -u -m pytest tests -q -x -m gpu --timeout 600 --timeout-method thread > gpurun_out/r02_c26/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "^FAILED|passed|failed" gpurun_out/r02_c26/pytest_gpu.log; tail -30 gpurun_out/r02_c26/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r02_c26/pytest_gpu.log
