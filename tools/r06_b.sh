#!/bin/bash
# gemm3e probe (A/B vs gemm3p and hipBLASLt, bitwise vs gemm3p), then the GPU suite and the
# spawned two-rank bench.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/g3e_probe.py > gpurun_out/r06b_g3e_probe.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06b_gpu_tests.log 2>&1
SRNN_DIST_BACKEND=gloo timeout -k 10 500 python3 bench.py --gpus 2 --steps 3 --warmup 2 --no-gen --no-cpu \
  > gpurun_out/r06b_spawn2.json 2> gpurun_out/r06b_spawn2.err
echo ok
