bash tools/gsteps.sh \
 "300 python -u -m pytest tests/test_gpu_kernels.py -k 'dtab or blocked' -v -s --timeout 120 --timeout-method thread > gpurun_out/r04d_dtab_tests.log 2>&1" \
 "400 python -u -m pytest tests/test_gpu_distributed.py -v -s --timeout 200 --timeout-method thread > gpurun_out/r04d_dp_tests.log 2>&1" \
 "600 python -u -m pytest tests/test_gpu_parity_big.py tests/test_gpu_parity.py -k 'big or _a or sampled or long or trajectory' -v -s --timeout 300 --timeout-method thread > gpurun_out/r04d_tests.log 2>&1"
