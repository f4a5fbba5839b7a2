#!/bin/bash
# Round-5 diagnosis of the in-launch tick GEMM: the bf16 generation identity test under each
# SRNN_GEN_TG_DBG mode (0 none, 1 drain every chunk wait, 2 agent acquire after the barrier).
mkdir -p gpurun_out
for d in 0 1 2 3; do
  SRNN_GEN_TG_DBG=$d timeout -k 10 120 python -u -m pytest tests/test_gpu_generation.py -m gpu -q --timeout 100 --timeout-method thread -k "bf16_d1024 and 128-1" > gpurun_out/r05_tgdbg_$d.log 2>&1
  rc=$?
  echo "dbg $d rc $rc: $(grep -E 'passed|failed' gpurun_out/r05_tgdbg_$d.log | tail -1)"
  grep -o "[0-9]* of [0-9]* draws differ" gpurun_out/r05_tgdbg_$d.log | head -1
  if [ $rc -gt 1 ]; then break; fi
done
