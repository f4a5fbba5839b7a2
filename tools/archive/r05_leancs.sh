#!/bin/bash
# Column-sum (da2) epilogue without bias / ReLU code: tests, lib A/B (ran from tools/)
set -e
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py -k "gemm or csum or colsum" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05cs_tests.log 2>&1
tail -1 gpurun_out/r05cs_tests.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05cs_tests2.log 2>&1
tail -1 gpurun_out/r05cs_tests2.log
TAG=r05cs COMBOS="A: B:" LAST=B ROUNDS=3 BS="512 64" SITES="'mlp_da2_gemm','mlp_da1_gemm'," bash tools/r05_combo.sh
