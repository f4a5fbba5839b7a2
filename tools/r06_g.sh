#!/bin/bash
# step kernel tables with and without the log-softmax epilogue (B = 512)
set -e
R=$PWD; O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
for v in 0 1; do
SRNN_LSM_EPI=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/p$v -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra > $O/r06g_prof_lsm$v.log 2>&1
db=$(find /tmp/p$v -name '*.db' | head -1)
python3 $R/tools/kstats.py $db 3 12 > $O/r06g_step_kernels_lsm$v.txt
done
echo ok
