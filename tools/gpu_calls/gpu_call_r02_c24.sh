set -o pipefail
mkdir -p gpurun_out/r02_c25
for v in "" ; do
  timeout -k 10 200 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -k "factor_f32_b32 or factor_f32_b16" > gpurun_out/r02_c25/pytest_$v.log 2>&1; echo "$v rc=$?"; tail -1 gpurun_out/r02_c25/pytest_$v.log
done
