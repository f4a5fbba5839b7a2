#!/bin/bash
# 64-row step (one row tile per sweep group): reverse-sweep operand loads nt (0, shipped) vs
# plain (SRNN_GX_EXP=512), alternated three times on one box
set -e
mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2 3; do for e in 0 512; do
  SRNN_GX_EXP=$e timeout -k 10 200 python3 bench.py --steps 30 --warmup 3 --no-gen --no-cpu --no-extra --batch 64 > gpurun_out/r06b64_${e}_$r.json 2> gpurun_out/r06b64_${e}_$r.err
  python3 -c "
import json
d=json.loads(open('gpurun_out/r06b64_${e}_$r.json').read().strip().splitlines()[-1])
print('exp $e round $r:', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d.get('kernels', {}).items() if 'gru' in k})
"
done; done
echo ok
