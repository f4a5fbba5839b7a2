#!/bin/bash
# log-softmax epilogue: tests, then A/B of the B = 512 step (SRNN_LSM_EPI=0 / 1, alternating)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm3e.py tests/test_gpu_bench_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06f_tests.log 2>&1
for i in 1 2; do
  for v in 0 1; do
    SRNN_LSM_EPI=$v timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra > gpurun_out/r06f_lsm${v}_$i.json 2> gpurun_out/r06f_lsm${v}_$i.err
  done
done
echo ok
