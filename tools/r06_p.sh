#!/bin/bash
# LDS-staged W_hh / W_hh^T fragment loads of the persistent GRU sweeps: the sweep tests, the
# sweep intercept probe, the bench's TBPTT lines
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_coresidency.py tests/test_gpu_bench_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gru or xcd or sweep or coresid or bench" > gpurun_out/r06p_tests.log 2>&1
timeout -k 10 240 python3 -u tools/gru_fixed_probe.py > gpurun_out/r06p_gru_fixed.txt 2>&1
timeout -k 10 300 python3 bench.py --no-gen --no-cpu > gpurun_out/r06p_bench.json 2> gpurun_out/r06p_bench.err
echo ok
