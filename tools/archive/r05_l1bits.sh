#!/bin/bash
# L1 gather's mask bits from the packed bf16 words: bits tests, then lib A/B (tools/r05_combo.sh)
set -e
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "bits or mlp_l1" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05l1_tests.log 2>&1
tail -1 gpurun_out/r05l1_tests.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "bits" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05l1_tests2.log 2>&1
tail -1 gpurun_out/r05l1_tests2.log
TAG=r05l1 COMBOS="A: B:" LAST=B ROUNDS=3 BS="512 64" SITES="'mlp_l1_gather','mlp_da1_gemm'," bash tools/r05_combo.sh
