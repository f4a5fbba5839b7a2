#!/bin/bash
# Grouped a1 mask bits (SRNN_A1_BITS): the bit-layout / GEMM / step parity tests, the da1 GEMM
# decomposition, then the step A/B (bench.py TBPTT lines, SRNN_A1_BITS=0/1 alternated).
set -e
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05a1}
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "bits" -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "bits" -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests2.log 2>&1
tail -1 gpurun_out/${TAG}_tests2.log
timeout -k 10 240 python3 tools/da1_probe.py > gpurun_out/${TAG}_da1_probe.txt 2>&1
cat gpurun_out/${TAG}_da1_probe.txt
TAG=${TAG}ab VAR=SRNN_A1_BITS SITES="'mlp_da1_gemm','dtab_scatter'," BS="512 64" ROUNDS=2 bash tools/r05_envab.sh
