# NN shapes on the ring ping-pong: GEMM tests, hand-written-only bench line, per-GEMM log
bash tools/gsteps.sh \
 "300 python -u -m pytest tests/test_gpu_kernels.py -k 'gemm' -q -rf --timeout 120 --timeout-method thread > gpurun_out/r04p_tests.log 2>&1" \
 "240 SRNN_BLASLT=0 python -u bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra > gpurun_out/r04p_hw_b512.json 2> gpurun_out/r04p_hw_b512.err" \
 "240 SRNN_BLASLT=0 SRNN_G3_NNQ=0 python -u bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra > gpurun_out/r04p_hw_b512_nnq0.json 2> gpurun_out/r04p_hw_b512_nnq0.err" \
 "240 python -u bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra > gpurun_out/r04p_b512.json 2> gpurun_out/r04p_b512.err"
