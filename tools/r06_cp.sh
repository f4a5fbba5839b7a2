#!/bin/bash
# dense activation casts: four-per-lane copy (SRNN_COPY_FLAT=1, new default) vs the element
# kernel (0); the cast tests first, then the step at 512 and 64 rows alternated on one box
set -e
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "cast_dense" -x -q --timeout 120 --timeout-method thread > gpurun_out/r06cp_tests.log 2>&1
tail -1 gpurun_out/r06cp_tests.log
for r in 1 2 3; do for b in 512 64; do for f in 0 1; do
  SRNN_COPY_FLAT=$f timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-gen --no-cpu --no-extra --batch $b > gpurun_out/r06cp_${b}_${f}_$r.json 2> gpurun_out/r06cp_${b}_${f}_$r.err
  python3 -c "
import json
d=json.loads(open('gpurun_out/r06cp_${b}_${f}_$r.json').read().strip().splitlines()[-1])
print('rows $b flat $f round $r:', d['ms_per_step'])
"
done; done; done
echo ok
