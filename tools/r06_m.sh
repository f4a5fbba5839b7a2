#!/bin/bash
# GEMM routing tests, then the bench's TBPTT lines at HEAD
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/r06m_tests.log 2>&1
timeout -k 10 300 python3 bench.py --no-gen --no-cpu > gpurun_out/r06m_bench.json 2> gpurun_out/r06m_bench.err
echo ok
