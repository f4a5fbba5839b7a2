#!/bin/bash
# Same-box A/B over library builds and env switches: COMBOS="B: B:SRNN_DTAB_PD=1 C: ..." runs
# each abso/lib_<X>.so with the given env (bench.py TBPTT lines only), ROUNDS alternations at
# each B; ms per step and the SITES' per-site times printed per run.  LAST stays in place.
set -e
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05cb}
LIB=jalil-saboorizadeh-multi-speaker-neural-vocoder_amd/libsamplernn_hip.so
for B in ${BS:-512 64}; do for r in $(seq 1 ${ROUNDS:-2}); do i=0; for c in $COMBOS; do
i=$((i+1)); v=${c%%:*}; e=${c#*:}
cp abso/lib_$v.so $LIB
env $e timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-gen --no-cpu --no-extra --batch $B > gpurun_out/${TAG}_b${B}_${i}_$r.json 2> gpurun_out/${TAG}_b${B}_${i}_$r.err
python3 -c "
import json
d=json.loads(open('gpurun_out/${TAG}_b${B}_${i}_$r.json').read().strip().splitlines()[-1])
ks=d.get('kernels',{})
print('B=$B $c round $r:', d['ms_per_step'], {k: ks[k].get('ms_per_step') for k in (${SITES:-'dtab_scatter',}) if k in ks})
"
done; done; done
cp abso/lib_${LAST:-B}.so $LIB
