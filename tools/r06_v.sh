#!/bin/bash
# reverse sweep, one row tile: next step's operands issued right after the hand-off lands
# (default) vs after the publish (SRNN_GX_EXP=256, same results); the sweep tests, the sweep
# probe in both forms and with the fetch skipped (64: timing only), the bench's TBPTT lines
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_coresidency.py tests/test_gpu_bench_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gru or xcd or sweep or coresid or bench" > gpurun_out/r06v_tests.log 2>&1
for e in 0 256 64; do
  SRNN_GX_EXP=$e timeout -k 10 240 python3 -u tools/gru_fixed_probe.py > gpurun_out/r06v_gru_exp$e.txt 2>&1
done
SRNN_GX_EXP=256 timeout -k 10 300 python3 bench.py --no-gen --no-cpu > gpurun_out/r06v_late.json 2> gpurun_out/r06v_late.err
timeout -k 10 300 python3 bench.py --no-gen --no-cpu > gpurun_out/r06v_early.json 2> gpurun_out/r06v_early.err
echo ok
