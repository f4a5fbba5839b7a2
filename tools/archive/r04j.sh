# GRU sweeps: early hand-off loads after the publish (MT > 1); tests then bench
bash tools/gsteps.sh \
 "300 python -u -m pytest tests/test_gpu_kernels.py -k 'gru_xcd' -v --timeout 120 --timeout-method thread > gpurun_out/r04j_tests.log 2>&1" \
 "240 python -u bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra > gpurun_out/r04j_b512.json 2> gpurun_out/r04j_b512.err" \
 "240 SRNN_DP_FORCE=1 SRNN_GRAPH=1 python -u tools/host_prof.py 64 10 > gpurun_out/r04j_host_prof_dp64.txt 2>&1"
