bash tools/gsteps.sh \
 "300 python -u -m pytest tests/test_gpu_kernels.py -k 'dtab or blocked' -x -v -s --timeout 120 --timeout-method thread > gpurun_out/r04b_dtab_tests.log 2>&1" \
 "500 python -u -m pytest tests/test_gpu_parity_big.py tests/test_gpu_parity.py -k 'big or _a or sampled or long or trajectory' -v -s --timeout 200 --timeout-method thread > gpurun_out/r04b_tests.log 2>&1" \
 "400 TAG=r04b BS='64 512' bash tools/prof_step.sh"
