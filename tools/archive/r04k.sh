# compile-time-D GRU forward, ZeRO opt-in: GRU + DP graph tests, bench A/B (poll sleep)
bash tools/gsteps.sh \
 "300 python -u -m pytest tests/test_gpu_kernels.py -k 'gru_xcd' -v --timeout 120 --timeout-method thread > gpurun_out/r04k_tests.log 2>&1" \
 "300 python -u -m pytest tests/test_gpu_distributed.py -k 'graph_captured' -v --timeout 200 --timeout-method thread > gpurun_out/r04k_dp_tests.log 2>&1" \
 "240 python -u bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra > gpurun_out/r04k_b512.json 2> gpurun_out/r04k_b512.err" \
 "240 SRNN_GX_DC=0 python -u bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra > gpurun_out/r04k_b512_dc0.json 2> gpurun_out/r04k_b512_dc0.err" \
 "240 SRNN_POLL_SLEEP=0 python -u bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra > gpurun_out/r04k_b512_ps0.json 2> gpurun_out/r04k_b512_ps0.err" \
 "240 python -u bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra > gpurun_out/r04k_b512b.json 2> gpurun_out/r04k_b512b.err"
