#!/bin/bash
# A/B of an environment switch on the generation loop: kernel means (rocprofv3 kernel trace of
# tools/gen_prof.py) and the bench's bf16 generation line, for VAR=0 and VAR=1.
#   bash tools/gen_ab.sh SRNN_SKINNY_NT
set -e
var=$1
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 0 1; do
  export $var=$v
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format rocpd -d /tmp/ab_$v -o run -- python3 $R/tools/gen_prof.py 128 40 > $R/gpurun_out/ab_$v.log 2>&1
  python3 $R/tools/rocpd_summary.py stats $(find /tmp/ab_$v -name '*.db' | head -1) 8 > $R/gpurun_out/ab_stats_$v.csv
  timeout -k 10 300 python3 $R/bench.py --no-cpu --no-gen-fp32 --no-gen-e --steps 2 --warmup 1 > $R/gpurun_out/ab_bench_$v.log 2>&1
done
echo done
