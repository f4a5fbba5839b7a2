#!/bin/bash
# Same-box A/B of an env switch on the TBPTT step: VAR=0/1 alternated ROUNDS times at each B
# (bench.py TBPTT lines only), ms per step printed per run.  TAG names the outputs.
set -e
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05env}
for B in ${BS:-64 512}; do for r in $(seq 1 ${ROUNDS:-2}); do for v in 0 1; do
env $VAR=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-gen --no-cpu --no-extra --batch $B > gpurun_out/${TAG}_b${B}_${v}_$r.json 2> gpurun_out/${TAG}_b${B}_${v}_$r.err
python3 -c "
import json
d=json.loads(open('gpurun_out/${TAG}_b${B}_${v}_$r.json').read().strip().splitlines()[-1])
ks=d.get('kernels',{})
print('B=$B $VAR=$v round $r:', d['ms_per_step'], {k: ks[k].get('ms_per_step') for k in (${SITES:-'dtab_scatter',}) if k in ks})
"
done; done; done
