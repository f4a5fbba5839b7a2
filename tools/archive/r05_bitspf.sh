#!/bin/bash
# grouped-bits da1 kernel with the unit-1 fragment prefetch (SRNN_G3_BITS_PF): tests with the
# switch on, then the step A/B (ran from tools/)
set -e
mkdir -p gpurun_out; export TMPDIR=/tmp
SRNN_G3_BITS_PF=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -k "bits" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05bp_tests.log 2>&1
tail -1 gpurun_out/r05bp_tests.log
TAG=r05bp VAR=SRNN_G3_BITS_PF SITES="'mlp_da1_gemm','mlp_da2_gemm'," BS="512 64" ROUNDS=3 bash tools/r05_envab.sh
