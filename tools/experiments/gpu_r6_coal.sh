#!/bin/bash
# Round 6: coalesced hand-over stores (gen_chain_asm.py COAL) — chain microbenchmark with and without,
# then parity of the engine with them and an A/B against the round-5 hand-over (libtqr_nocoal.so).
set -o pipefail
O=gpurun_out/${1:-r6coal}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 tools/ubench/chain_asm_bench_nocoal 96 2 > $O/ubench_nocoal.txt 2>&1 || exit 1
timeout -k 10 120 tools/ubench/chain_asm_bench 96 2 > $O/ubench_coal.txt 2>&1 || exit 1
cat $O/ubench_nocoal.txt $O/ubench_coal.txt
PYTEST_FILES=tests/test_gpu_factor.py PYTEST_K="test_factor_vs_oracle or c3 or order or structured" BASE=libtqr_nocoal.so \
  BENCH_ARGS=--no-single-leg bash tools/gpu_ab_round.sh ${1:-r6coal}/ab libtqr.so 3
