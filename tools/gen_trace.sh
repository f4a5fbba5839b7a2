#!/bin/bash
# Kernel traces of one generation call (128 rows x N cond rows, dim 1024) per dtype:
#   bash tools/gen_trace.sh [N]  -> gpurun_out/gen_trace_<dtype>.txt (per-kernel totals per call)
set -e
R=$PWD; O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
n=${1:-100}
for dt in bf16 fp32; do
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d /tmp/gt_$dt -o run -- python3 $R/tools/gen_prof.py $dt $n > $O/gen_trace_$dt.log 2>&1
f=$(find /tmp/gt_$dt -name '*kernel_trace.csv' | head -1)
python3 $R/tools/trace_summary.py $f 2 30 > $O/gen_trace_$dt.txt
done
