bash tools/gsteps.sh \
 "200 python -u -m pytest tests/test_gpu_kernels.py -k 'nonfinite or skew' -v -s --timeout 120 --timeout-method thread > gpurun_out/r04e_dtab_tests.log 2>&1" \
 "300 python -u -m pytest tests/test_gpu_parity_big.py -k 'sampled' -v -s --timeout 300 --timeout-method thread > gpurun_out/r04e_tests.log 2>&1" \
 "300 python -u -m pytest tests/test_gpu_distributed.py -k 'graph_captured or bf16_buckets' -v -s --timeout 200 --timeout-method thread > gpurun_out/r04e_dp_tests.log 2>&1" \
 "400 TAG=r04e BS='64' bash tools/prof_step.sh"
