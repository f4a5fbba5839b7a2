# per-GEMM timings at 64 rows (the 8-GPU share): shipped routing vs hand-written only
bash tools/gsteps.sh \
 "240 SRNN_GRAPH=0 SRNN_GEMM_LOG=1 python -u bench.py --steps 2 --warmup 1 --no-gen --no-cpu --no-extra --batch 64 > gpurun_out/r04u_gemmlog64.json 2> gpurun_out/r04u_gemmlog64.err" \
 "240 SRNN_BLASLT=0 SRNN_GRAPH=0 SRNN_GEMM_LOG=1 python -u bench.py --steps 2 --warmup 1 --no-gen --no-cpu --no-extra --batch 64 > gpurun_out/r04u_gemmlog64_hw.json 2> gpurun_out/r04u_gemmlog64_hw.err" \
 "240 SRNN_GRAPH=0 SRNN_GEMM_LOG=1 python -u bench.py --steps 2 --warmup 1 --no-gen --no-cpu --no-extra --batch 128 > gpurun_out/r04u_gemmlog128.json 2> gpurun_out/r04u_gemmlog128.err" \
 "240 SRNN_BLASLT=0 SRNN_GRAPH=0 SRNN_GEMM_LOG=1 python -u bench.py --steps 2 --warmup 1 --no-gen --no-cpu --no-extra --batch 128 > gpurun_out/r04u_gemmlog128_hw.json 2> gpurun_out/r04u_gemmlog128_hw.err"
