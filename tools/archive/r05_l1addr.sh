#!/bin/bash
# L1 gather table-read addresses as one shift-add: tests, lib A/B (ran from tools/)
set -e
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "mlp_l1 or bits" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05la_tests.log 2>&1
tail -1 gpurun_out/r05la_tests.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_parity.py tests/test_gpu_parity_big.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05la_tests2.log 2>&1
tail -1 gpurun_out/r05la_tests2.log
TAG=r05la COMBOS="A: B:" LAST=B ROUNDS=3 BS="512 64" SITES="'mlp_l1_gather','mlp_da1_gemm'," bash tools/r05_combo.sh
