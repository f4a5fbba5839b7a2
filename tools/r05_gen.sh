#!/bin/bash
# Round-5 generation check: the generation tests, then the bench's generation lines only
# (TAG names the outputs), then a rocprofv3 kernel trace of a short bf16 generation.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r05g}
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_generation.py} -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu --no-extra --batch 64 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
echo ok
