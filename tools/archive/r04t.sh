# hipBLASLt candidate timing (SRNN_BLASLT_TUNE=n): GEMM tests with it on, then a bench A/B
B="python -u bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra"
bash tools/gsteps.sh \
 "300 SRNN_BLASLT_TUNE=16 python -u -m pytest tests/test_gpu_kernels.py -k 'blaslt' -q -rf --timeout 120 --timeout-method thread > gpurun_out/r04t_tests.log 2>&1" \
 "240 $B > gpurun_out/r04t_0.json 2> gpurun_out/r04t_0.err" \
 "240 SRNN_BLASLT_TUNE=16 $B > gpurun_out/r04t_16.json 2> gpurun_out/r04t_16.err" \
 "240 $B > gpurun_out/r04t_0b.json 2> gpurun_out/r04t_0b.err" \
 "240 SRNN_BLASLT_TUNE=16 $B > gpurun_out/r04t_16b.json 2> gpurun_out/r04t_16b.err" \
 "300 SRNN_BLASLT_TUNE=16 TAG=r04t BS='512' bash tools/prof_step.sh"
