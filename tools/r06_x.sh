#!/bin/bash
# reverse sweep operand fetch: order (post-MFMA vs after the publish, bit 256) x cache policy
# (nt streaming vs plain, bit 512); the sweep tests first
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_bench_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gru or xcd or sweep or bench" > gpurun_out/r06x_tests.log 2>&1
for e in 0 256 512 768; do
  SRNN_GX_EXP=$e timeout -k 10 240 python3 -u tools/gru_fixed_probe.py > gpurun_out/r06x_gru_exp$e.txt 2>&1
done
echo ok
