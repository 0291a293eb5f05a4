#!/bin/bash
# Multi-rank engine probe on ONE GPU: N ranks (torch.distributed.run, gloo), each with a share of
# the CUs (TQR_FLOW_GRID), tests/dist_worker.py at growing sizes; stops at the first failure.
# Each config is "m n b grid nproc" (nproc defaults to 2). Output: gpurun_out/dist/probe.log.
set -o pipefail
mkdir -p gpurun_out/dist
if [ -n "$DIST_CFGS" ]; then IFS=';' read -ra CFGS <<< "$DIST_CFGS"; else
  CFGS=("4096 4096 256 96" "16384 4096 256 96" "32768 8192 256 96" "32768 8192 256 128" "16384 4096 256 60 4" "8192 4096 256 30 8")
fi
for cfg in "${CFGS[@]}"; do
  set -- $cfg
  np=${5:-2}
  echo "== m=$1 n=$2 b=$3 grid=$4 ranks=$np" | tee -a gpurun_out/dist/probe.log
  TQR_FLOW_GRID=$4 timeout -k 10 150 python -m torch.distributed.run --nproc-per-node $np --master-addr 127.0.0.1 \
    --master-port 29512 tests/dist_worker.py $1 $2 $3 f64 0 >> gpurun_out/dist/probe.log 2>&1
  rc=$?
  echo "rc $rc" | tee -a gpurun_out/dist/probe.log
  [ $rc = 0 ] || break
done
