#!/bin/bash
# generation: the tick GEMM's weight rows and the resident fragment images as plain
# (abso/lib_A.so) vs non-temporal loads (abso/lib_N.so, -DSRNN_GEN_NT=1), alternated on one
# box; the bench's generation lines (a short 64-row TBPTT part runs first)
set -e
mkdir -p gpurun_out; export TMPDIR=/tmp
LIB=jalil-saboorizadeh-multi-speaker-neural-vocoder_amd/libsamplernn_hip.so
for r in 1 2; do for v in A N; do
  cp abso/lib_$v.so $LIB
  timeout -k 10 300 python3 bench.py --steps 3 --warmup 2 --no-cpu --no-extra --batch 64 > gpurun_out/r06gnt_${v}_$r.json 2> gpurun_out/r06gnt_${v}_$r.err
  python3 -c "
import json
d=json.loads(open('gpurun_out/r06gnt_${v}_$r.json').read().strip().splitlines()[-1])
print('$v round $r:', {k: (d[k]['x_realtime'], d[k]['us_per_step']) for k in ('gen', 'gen_fp32', 'gen_config_e', 'gen_config_e_fp32') if k in d})
"
done; done
cp abso/lib_A.so $LIB
echo ok
