set -o pipefail
mkdir -p gpurun_out/r02_c31
timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-api > gpurun_out/r02_c31/bench.json 2> gpurun_out/r02_c31/bench.err || { echo bench failed; tail gpurun_out/r02_c31/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r02_c31/bench.json').read());print('f64', d['ms_per_step'], d['roofline']['frac'], d.get('status'))"
TQR_FST_LIB=libtqr_fst.so timeout -k 10 200 python tools/flowstamps.py 16384 > gpurun_out/r02_c31/fst.txt 2>&1 || { echo "fst failed"; tail gpurun_out/r02_c31/fst.txt; exit 1; }
grep -E "wall|phase|drain|barrier|wave" gpurun_out/r02_c31/fst.txt
