#!/bin/bash
# register-resident conv_t weight-norm backward: its bit-exactness tests, the TBPTT tests,
# then the bench's TBPTT lines with it off (SRNN_WN_REG=0) and on
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity_big.py tests/test_gpu_bench_parity.py tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -k "convt or weight_norm or wn or tbptt or bench" > gpurun_out/r06t_tests.log 2>&1
SRNN_WN_REG=0 timeout -k 10 300 python3 bench.py --no-gen --no-cpu > gpurun_out/r06t_off.json 2> gpurun_out/r06t_off.err
timeout -k 10 300 python3 bench.py --no-gen --no-cpu > gpurun_out/r06t_on.json 2> gpurun_out/r06t_on.err
echo ok
