#!/bin/bash
# Re-entry pass at HEAD: the GPU suite, bench.py --gpus 2 WITHOUT torchrun (the parent spawns
# both ranks; gloo, both on the one GPU: a rehearsal, not a performance number), default bench.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06i_gpu_tests.log 2>&1
SRNN_DIST_BACKEND=gloo timeout -k 10 500 python3 bench.py --gpus 2 --steps 3 --warmup 2 --no-gen --no-cpu \
  > gpurun_out/r06i_spawn2.json 2> gpurun_out/r06i_spawn2.err
timeout -k 10 400 python3 bench.py > gpurun_out/r06i_bench.json 2> gpurun_out/r06i_bench.err
echo ok
