# per-GEMM timings with every GEMM on gemm3 in each of its schedules (ring/pair default, ping-pong, q)
bash tools/gsteps.sh \
 "240 SRNN_G3MODE=3 SRNN_BLASLT=0 SRNN_GRAPH=0 SRNN_GEMM_LOG=1 python -u bench.py --steps 2 --warmup 1 --no-gen --no-cpu --no-extra > gpurun_out/r04o_gemmlog_m3.json 2> gpurun_out/r04o_gemmlog_m3.err" \
 "240 SRNN_G3MODE=4 SRNN_BLASLT=0 SRNN_GRAPH=0 SRNN_GEMM_LOG=1 python -u bench.py --steps 2 --warmup 1 --no-gen --no-cpu --no-extra > gpurun_out/r04o_gemmlog_m4.json 2> gpurun_out/r04o_gemmlog_m4.err" \
 "240 SRNN_G3MODE=1 SRNN_BLASLT=0 SRNN_GRAPH=0 SRNN_GEMM_LOG=1 python -u bench.py --steps 2 --warmup 1 --no-gen --no-cpu --no-extra > gpurun_out/r04o_gemmlog_m1.json 2> gpurun_out/r04o_gemmlog_m1.err"
