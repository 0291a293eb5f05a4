export TQR_FLOW_SHAPE=r
timeout -k 10 300 python -u -m pytest tests/test_gpu_factor.py -x -v --timeout 120 --timeout-method thread -k "test_factor_vs_oracle and 256 and float64" > gpurun_out/res1.log 2>&1; rc=$?
tail -5 gpurun_out/res1.log
exit $rc
