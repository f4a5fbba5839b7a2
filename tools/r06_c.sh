#!/bin/bash
# gemm3e after the piece-swizzle fix: bitwise tests vs gemm3p, then the A/B probe
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm3e.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06c_g3e_tests.log 2>&1
timeout -k 10 300 python3 -u tools/g3e_probe.py > gpurun_out/r06c_g3e_probe.txt 2>&1
echo ok
