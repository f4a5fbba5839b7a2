#!/bin/bash
# A change's check: the named -m gpu tests (TESTS, pytest args), then the 512- and 64-row
# steps (bench.py TBPTT lines only).  TAG names the outputs under gpurun_out/.
set -e
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05ab}
timeout -k 10 ${TT:-600} python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
tail -1 gpurun_out/${TAG}_tests.log
for B in ${BS:-512 64}; do
timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra --batch $B > gpurun_out/${TAG}_b$B.json 2> gpurun_out/${TAG}_b$B.err
python3 -c "
import json
d=json.loads(open('gpurun_out/${TAG}_b$B.json').read().strip().splitlines()[-1])
print($B, d['ms_per_step'])
"
done
