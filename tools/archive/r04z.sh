# da2 GEMM epilogue column sums (hidden bias gradient): kernel + parity + graph tests, bench A/B
B="python -u bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra"
bash tools/gsteps.sh \
 "300 python -u -m pytest tests/test_gpu_kernels.py -k 'csum or amax or gemm3' -q -rf --timeout 120 --timeout-method thread > gpurun_out/r04z_kern.log 2>&1" \
 "400 python -u -m pytest tests/test_gpu_bench_parity.py tests/test_gpu_graph.py -q -rf -s --timeout 300 --timeout-method thread > gpurun_out/r04z_parity.log 2>&1" \
 "240 $B > gpurun_out/r04z_on.json 2> gpurun_out/r04z_on.err" \
 "240 SRNN_CSUM_EPI=0 $B > gpurun_out/r04z_off.json 2> gpurun_out/r04z_off.err" \
 "240 $B > gpurun_out/r04z_on2.json 2> gpurun_out/r04z_on2.err" \
 "240 SRNN_CSUM_EPI=0 $B > gpurun_out/r04z_off2.json 2> gpurun_out/r04z_off2.err"
