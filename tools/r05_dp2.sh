#!/bin/bash
# Two-rank rehearsal on ONE GPU (gloo; both ranks on device 0) with the extra lines (weak_64,
# weak_512): distributed.init declares the shared device, so each rank's persistent sweeps are
# sized to half the CUs (csrc/handoff.hpp co-residency) -- the round-4 weak_512 spin-out
# (profiles/r04_dp2_rehearsal_303edb90.err.txt) must not recur.  Not a performance number.
set -e
mkdir -p gpurun_out
TAG=${TAG:-r05_dp2}
SRNN_DIST_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 2 --no-gen --no-cpu \
  > gpurun_out/${TAG}.json 2> gpurun_out/${TAG}.err
echo ok
