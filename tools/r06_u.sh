#!/bin/bash
# timing-only switches of the reverse sweep (results invalid): per-step cost without the
# next step's operand fetch (SRNN_GX_EXP=64), without the output stores (1), without both (65)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for e in 0 64 1 65; do
  SRNN_GX_EXP=$e timeout -k 10 240 python3 -u tools/gru_fixed_probe.py > gpurun_out/r06u_gru_exp$e.txt 2>&1
done
echo ok
