# per-GEMM timings of one eager B = 512 step with every GEMM on the hand-written kernels
bash tools/gsteps.sh \
 "240 SRNN_BLASLT=0 SRNN_GRAPH=0 SRNN_GEMM_LOG=1 python -u bench.py --steps 2 --warmup 1 --no-gen --no-cpu --no-extra > gpurun_out/r04n_gemmlog_hw.json 2> gpurun_out/r04n_gemmlog_hw.err" \
 "240 SRNN_GRAPH=0 SRNN_GEMM_LOG=1 python -u bench.py --steps 2 --warmup 1 --no-gen --no-cpu --no-extra > gpurun_out/r04n_gemmlog.json 2> gpurun_out/r04n_gemmlog.err"
