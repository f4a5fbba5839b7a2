#!/bin/bash
# Per-step kernel tables of the timed graph replays (run from the repo root on the GPU box):
#   TAG=r03b BS="512 128" bash tools/prof_step.sh
# -> gpurun_out/<tag>_step_kernels_b<B>.txt (tools/kstats.py over rocprofv3 --kernel-trace --stats)
set -e
R=$PWD; O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
TAG=${TAG:-r03}
for B in ${BS:-512 128}; do
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/p$B -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra --batch $B > $O/${TAG}_prof_b$B.log 2>&1
db=$(find /tmp/p$B -name '*.db' | head -1)
python3 $R/tools/kstats.py $db 3 12 --sequence > $O/${TAG}_step_kernels_b$B.txt
cp $(find /tmp/p$B -name '*kernel_stats.csv' | head -1) $O/${TAG}_kernel_stats_b$B.csv || true
done
