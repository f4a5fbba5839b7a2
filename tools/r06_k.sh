#!/bin/bash
# GEMM routing probe of the TBPTT step at 64 and 512 rows (tools/gemm_route_probe.py)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/gemm_route_probe.py --rows 64 > gpurun_out/r06k_route_b64.txt 2> gpurun_out/r06k_route_b64.err
timeout -k 10 400 python3 -u tools/gemm_route_probe.py --rows 512 --reps 5 > gpurun_out/r06k_route_b512.txt 2> gpurun_out/r06k_route_b512.err
echo ok
