# bias-gradient column sums on a side stream: graph / parity / DP tests, then bench A/B
bash tools/gsteps.sh \
 "400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_bench_parity.py tests/test_gpu_distributed.py tests/test_gpu_parity_big.py -q -rf --timeout 300 --timeout-method thread > gpurun_out/r04l_tests.log 2>&1" \
 "240 python -u bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra > gpurun_out/r04l_b512.json 2> gpurun_out/r04l_b512.err" \
 "240 SRNN_SIDE_STREAM=0 python -u bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra > gpurun_out/r04l_b512_s0.json 2> gpurun_out/r04l_b512_s0.err" \
 "240 python -u bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra --batch 64 > gpurun_out/r04l_b64.json 2> gpurun_out/r04l_b64.err" \
 "240 SRNN_SIDE_STREAM=0 python -u bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra --batch 64 > gpurun_out/r04l_b64_s0.json 2> gpurun_out/r04l_b64_s0.err"
