#!/bin/bash
# Per-step kernel tables of the DP step on one GPU (forced one-rank RCCL group, graph mode):
# ZeRO-1 on and off, 64 rows.  -> gpurun_out/<TAG>_dp_{zero,nozero}_kernels.txt
set -e
R=$PWD; O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
TAG=${TAG:-r04}
for Z in 1 0; do
n=$([ $Z = 1 ] && echo zero || echo nozero)
SRNN_DP_FORCE=1 SRNN_DP_ZERO=$Z timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/d$Z -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra --batch 64 > $O/${TAG}_dp_${n}_prof.log 2>&1
db=$(find /tmp/d$Z -name '*.db' | head -1)
python3 $R/tools/kstats.py $db 3 12 --sequence > $O/${TAG}_dp_${n}_kernels.txt
done
