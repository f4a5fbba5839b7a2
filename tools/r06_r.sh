#!/bin/bash
# batched hipBLASLt (the folded table build): GEMM tests, generation tests (bf16 table too),
# the bench's TBPTT lines, the 64-row step table
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_generation.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06r_tests.log 2>&1
timeout -k 10 300 python3 bench.py --no-gen --no-cpu > gpurun_out/r06r_bench.json 2> gpurun_out/r06r_bench.err
TAG=r06r BS="64" bash tools/prof_step.sh
echo ok
