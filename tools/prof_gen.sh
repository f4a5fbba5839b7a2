#!/bin/bash
# Kernel timeline of configs[2] generation (128 rows, dim 1024) per dtype:
#   TAG=r04 DTS="bf16 fp32" bash tools/prof_gen.sh
# -> gpurun_out/<tag>_gen_kernels_<dt>.txt: kstats over 8 persistent launches (two top-tier
#    periods) in the steady state, with the launch-order sequence of the first period.
set -e
R=$PWD; O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
for DT in ${DTS:-bf16 fp32}; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/g$DT -o run -- python3 $R/tools/gen_prof.py $DT 40 > $O/${TAG}_gen_prof_$DT.log 2>&1
db=$(find /tmp/g$DT -name '*.db' | head -1)
python3 $R/tools/kstats.py $db 60 67 --marker gen_mlp_kernel --sequence --span 4 > $O/${TAG}_gen_kernels_$DT.txt
done
