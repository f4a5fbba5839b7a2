#!/bin/bash
# Routing change A/B: the probe at the new default route (64 / 512 rows), then the bench's
# TBPTT lines with the round-6 routing off (SRNN_BLASLT_WIDE_K=0 SRNN_SMALLK_G3=0) and on,
# alternated twice on the same box
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/gemm_route_probe.py --rows 64 > gpurun_out/r06l_route_b64.txt 2> gpurun_out/r06l_route_b64.err
timeout -k 10 400 python3 -u tools/gemm_route_probe.py --rows 512 --reps 5 > gpurun_out/r06l_route_b512.txt 2> gpurun_out/r06l_route_b512.err
for r in 1 2; do
  SRNN_BLASLT_WIDE_K=0 SRNN_SMALLK_G3=0 timeout -k 10 300 python3 bench.py --no-gen --no-cpu > gpurun_out/r06l_off$r.json 2> gpurun_out/r06l_off$r.err
  timeout -k 10 300 python3 bench.py --no-gen --no-cpu > gpurun_out/r06l_on$r.json 2> gpurun_out/r06l_on$r.err
done
echo ok
