#!/bin/bash
# GRU sweep changes: the sweep / parity tests, then the 512- and 64-row steps (bench.py's
# gru_sweep microbench and probed sites).  TAG names the outputs.
set -e
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05x}
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "xcd or gru_seq" tests/test_gpu_coresidency.py tests/test_gpu_bench_parity.py tests/test_gpu_graph.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
for B in 512 64; do
timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra --batch $B > gpurun_out/${TAG}_b$B.json 2> gpurun_out/${TAG}_b$B.err
python3 -c "
import json
d=json.loads(open('gpurun_out/${TAG}_b$B.json').read().strip().splitlines()[-1])
print($B, d['ms_per_step'], d['gru_sweep']['fwd']['us_per_step'], d['gru_sweep']['bwd']['us_per_step'], {k:v.get('ms_per_step') for k,v in d['kernels'].items() if 'gru' in k})
"
done
