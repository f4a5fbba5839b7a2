#!/bin/bash
# persistent GRU sweeps: non-temporal operand loads (bit 512 off) and output stores (bit 2048
# off) vs plain; the sweep tests, the sweep probe in four forms, the bench's TBPTT lines
# with all plain (2560, the round-5 form) and all nt (0)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_coresidency.py tests/test_gpu_bench_parity.py tests/test_gpu_persistent_errors.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gru or xcd or sweep or coresid or bench or persist" > gpurun_out/r06y_tests.log 2>&1
for e in 0 512 2048 2560; do
  SRNN_GX_EXP=$e timeout -k 10 240 python3 -u tools/gru_fixed_probe.py > gpurun_out/r06y_gru_exp$e.txt 2>&1
done
SRNN_GX_EXP=2560 timeout -k 10 300 python3 bench.py --no-gen --no-cpu > gpurun_out/r06y_plain.json 2> gpurun_out/r06y_plain.err
timeout -k 10 300 python3 bench.py --no-gen --no-cpu > gpurun_out/r06y_nt.json 2> gpurun_out/r06y_nt.err
echo ok
