#!/bin/bash
# Lean grouped-bits epilogue (da1): GEMM / bits / step parity tests, da1 probe, lib A/B
set -e
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py -k "bits or gemm or dtab" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05ln_tests.log 2>&1
tail -1 gpurun_out/r05ln_tests.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05ln_tests2.log 2>&1
tail -1 gpurun_out/r05ln_tests2.log
timeout -k 10 240 python3 tools/da1_probe.py > gpurun_out/r05ln_da1_probe.txt 2>&1
head -3 gpurun_out/r05ln_da1_probe.txt
TAG=r05ln COMBOS="A: B:" LAST=B ROUNDS=3 BS="512 64" SITES="'mlp_da1_gemm','dtab_scatter'," bash tools/r05_combo.sh
