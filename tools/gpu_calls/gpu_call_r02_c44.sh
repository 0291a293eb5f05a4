set -o pipefail
mkdir -p gpurun_out/r02_c44
timeout -k 10 300 python tools/tile_bench.py 2048 > gpurun_out/r02_c44/tile_bench.jsonl 2> gpurun_out/r02_c44/tile_bench.err || { echo tile bench failed; tail gpurun_out/r02_c44/tile_bench.err; exit 1; }
cat gpurun_out/r02_c44/tile_bench.jsonl
