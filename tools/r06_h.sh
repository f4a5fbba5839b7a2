#!/bin/bash
# the GPU suite at HEAD, then bench.py --gpus 2 WITHOUT torchrun (the parent spawns both
# ranks; gloo, both on the one GPU: a rehearsal, not a performance number)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06h_gpu_tests.log 2>&1
SRNN_DIST_BACKEND=gloo timeout -k 10 500 python3 bench.py --gpus 2 --steps 3 --warmup 2 --no-gen --no-cpu \
  > gpurun_out/r06h_spawn2.json 2> gpurun_out/r06h_spawn2.err
echo ok
