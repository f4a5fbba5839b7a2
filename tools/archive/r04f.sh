bash tools/gsteps.sh \
 "300 python -u -m pytest tests/test_gpu_parity_big.py -k 'sampled' -v -s --timeout 300 --timeout-method thread > gpurun_out/r04f_tests.log 2>&1" \
 "300 python -u -m pytest tests/test_gpu_distributed.py -k 'graph_captured' -v -s --timeout 200 --timeout-method thread > gpurun_out/r04f_dp_tests.log 2>&1" \
 "450 TAG=r04f DTS='bf16 fp32' bash tools/prof_gen.sh"
