set -o pipefail
mkdir -p gpurun_out/r02_c28
timeout -k 10 400 python -u -m pytest tests -q -x -m gpu --timeout 300 --timeout-method thread -k "not 65536 and not 32768" > gpurun_out/r02_c28/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "^FAILED|passed|failed" gpurun_out/r02_c28/pytest_gpu.log; tail -30 gpurun_out/r02_c28/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r02_c28/pytest_gpu.log
timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-api > gpurun_out/r02_c28/bench.json 2> gpurun_out/r02_c28/bench.err || { echo bench failed; tail gpurun_out/r02_c28/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r02_c28/bench.json').read());print('f64', d['ms_per_step'], d['roofline']['frac'])"
TQR_FST_LIB=libtqr_fst.so timeout -k 10 200 python tools/flowstamps.py 16384 > gpurun_out/r02_c28/fst.txt 2>&1 || { echo "fst failed"; tail gpurun_out/r02_c28/fst.txt; exit 1; }
grep -E "wall|phase|drain|barrier|head|strip|W \+" gpurun_out/r02_c28/fst.txt
