#!/bin/bash
# Two-rank rehearsal of bench.py's data-parallel path on ONE GPU (gloo backend; both ranks on
# device 0, 256 rows each = configs[3] at N = 2): GradAllReduce hooks, deferred bucket launches,
# sweep fences and the lagged failure check with the bf16 model.  Not a performance number
# (gloo moves the buckets through host memory; the two ranks share the GPU).
set -e
mkdir -p gpurun_out
SRNN_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 2 --no-gen --no-cpu --no-extra \
  > gpurun_out/r03c_dp2_rehearsal.json 2> gpurun_out/r03c_dp2_rehearsal.err
echo ok
