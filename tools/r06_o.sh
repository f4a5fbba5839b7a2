#!/bin/bash
# thin-N GEMM tests + probe after the pipelining; GRU sweep intercepts with / without the reverse
# sweep's W_hh^T fragment loads (SRNN_GX_EXP=128, timing only)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "small or thin or gemm_n or route" > gpurun_out/r06o_tests.log 2>&1
timeout -k 10 400 python3 -u tools/gemm_route_probe.py --rows 512 --reps 5 > gpurun_out/r06o_route_b512.txt 2> gpurun_out/r06o_route_b512.err
timeout -k 10 240 python3 -u tools/gru_fixed_probe.py > gpurun_out/r06o_gru_fixed.txt 2>&1
SRNN_GX_EXP=128 timeout -k 10 240 python3 -u tools/gru_fixed_probe.py > gpurun_out/r06o_gru_fixed_exp128.txt 2>&1
echo ok
