# packed saved gates in the XCD GRU sweeps: kernel tests, TBPTT parity, bench A/B
B="python -u bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra"
bash tools/gsteps.sh \
 "300 python -u -m pytest tests/test_gpu_kernels.py -k 'gru' -q -rf --timeout 120 --timeout-method thread > gpurun_out/r04x_tests.log 2>&1" \
 "400 python -u -m pytest tests/test_gpu_bench_parity.py tests/test_gpu_graph.py tests/test_gpu_parity_big.py -k 'not persistent_fp32_long' -q -rf --timeout 300 --timeout-method thread > gpurun_out/r04x_parity.log 2>&1" \
 "240 $B > gpurun_out/r04x_b512.json 2> gpurun_out/r04x_b512.err" \
 "240 SRNN_GX_GPK=0 $B > gpurun_out/r04x_b512_0.json 2> gpurun_out/r04x_b512_0.err" \
 "240 $B --batch 64 > gpurun_out/r04x_b64.json 2> gpurun_out/r04x_b64.err" \
 "240 SRNN_GX_GPK=0 $B --batch 64 > gpurun_out/r04x_b64_0.json 2> gpurun_out/r04x_b64_0.err" \
 "150 SRNN_GRU_DIAG=1 python -u tools/archive/gru_stamp_probe.py 512 > gpurun_out/r04x_gru512.txt 2>&1" \
 "150 SRNN_GRU_DIAG=1 python -u tools/archive/gru_stamp_probe.py 128 > gpurun_out/r04x_gru128.txt 2>&1"
