#!/bin/bash
# Same-box A/B of two builds of the library: abso/lib_A.so (before) and abso/lib_B.so (after)
# swapped in turn into the package, ROUNDS alternations at each B (bench.py TBPTT lines only);
# ms per step and the SITES' per-site times printed per run (VARIANTS picks the lib_X.so; LAST stays).
set -e
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05so}
LIB=jalil-saboorizadeh-multi-speaker-neural-vocoder_amd/libsamplernn_hip.so
for B in ${BS:-512 64}; do for r in $(seq 1 ${ROUNDS:-2}); do for v in ${VARIANTS:-A B}; do
cp abso/lib_$v.so $LIB
timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-gen --no-cpu --no-extra --batch $B > gpurun_out/${TAG}_b${B}_${v}_$r.json 2> gpurun_out/${TAG}_b${B}_${v}_$r.err
python3 -c "
import json
d=json.loads(open('gpurun_out/${TAG}_b${B}_${v}_$r.json').read().strip().splitlines()[-1])
ks=d.get('kernels',{})
print('B=$B lib=$v round $r:', d['ms_per_step'], {k: ks[k].get('ms_per_step') for k in (${SITES:-'dtab_scatter',}) if k in ks})
"
done; done; done
cp abso/lib_${LAST:-B}.so $LIB
