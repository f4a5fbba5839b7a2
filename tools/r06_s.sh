#!/bin/bash
# checkpoint at HEAD: the whole GPU suite, smoke, the default bench line
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06s_gpu_tests.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06s_smoke.log 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/r06s_bench.json 2> gpurun_out/r06s_bench.err
echo ok
