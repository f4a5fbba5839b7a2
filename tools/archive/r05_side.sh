#!/bin/bash
# Side-stream backward: the touched -m gpu tests, then 64 / 512-row steps with SRNN_SIDE=0 / 1.
set -e
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05s}
timeout -k 10 ${TT:-700} python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_bench_parity.py tests/test_gpu_graph.py tests/test_gpu_custom_ops.py tests/test_gpu_distributed.py tests/test_gpu_parity_big.py} -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
for B in ${BS:-64 512}; do for S in 0 1; do
SRNN_SIDE=$S timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-gen --no-cpu --no-extra --batch $B > gpurun_out/${TAG}_b${B}_side$S.json 2> gpurun_out/${TAG}_b${B}_side$S.err
done; done
grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/${TAG}_b*_side*.json
