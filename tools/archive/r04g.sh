# dTab blocked-copy A/B at B = 512 and the DP step at 64 rows (one-rank RCCL group, forced):
# eager vs graph-captured, ZeRO-1 on.
B="python -u bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra"
bash tools/gsteps.sh \
 "240 SRNN_DTAB_BLK=0 $B > gpurun_out/r04g_blk0.json 2> gpurun_out/r04g_blk0.err" \
 "240 SRNN_DTAB_BLK=1 $B > gpurun_out/r04g_blk1.json 2> gpurun_out/r04g_blk1.err" \
 "240 SRNN_DTAB_BLK=0 $B > gpurun_out/r04g_blk0b.json 2> gpurun_out/r04g_blk0b.err" \
 "240 SRNN_DTAB_BLK=1 $B > gpurun_out/r04g_blk1b.json 2> gpurun_out/r04g_blk1b.err" \
 "240 $B --batch 64 > gpurun_out/r04g_b64.json 2> gpurun_out/r04g_b64.err" \
 "240 SRNN_DP_FORCE=1 SRNN_GRAPH_DP=0 $B --batch 64 > gpurun_out/r04g_dp_eager.json 2> gpurun_out/r04g_dp_eager.err" \
 "240 SRNN_DP_FORCE=1 $B --batch 64 > gpurun_out/r04g_dp_graph.json 2> gpurun_out/r04g_dp_graph.err" \
 "240 SRNN_DP_FORCE=1 SRNN_DP_ZERO=0 $B --batch 64 > gpurun_out/r04g_dp_graph_nozero.json 2> gpurun_out/r04g_dp_graph_nozero.err" \
 "240 SRNN_GRAPH=0 SRNN_GEMM_LOG=1 python -u bench.py --steps 2 --warmup 1 --no-gen --no-cpu --no-extra > gpurun_out/r04g_gemmlog.json 2> gpurun_out/r04g_gemmlog.err"
