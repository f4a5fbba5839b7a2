#!/bin/bash
# HBM traffic of the bf16 generation loop, two separate rocprofv3 --pmc passes:
#   TAG=r04 bash tools/pmc_gen.sh  ->  gpurun_out/<TAG>_pmc_gen.txt (copy to profiles/)
set -e
R=$PWD; O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
cmd="python3 $R/tools/gen_prof.py bf16 20"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d /tmp/gf -o run -- $cmd > $O/pmc_gen_f.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d /tmp/gw -o run -- $cmd > $O/pmc_gen_w.log 2>&1
python3 $R/tools/pmc_gen.py $(find /tmp/gf -name '*.db' | head -1) $(find /tmp/gw -name '*.db' | head -1) > $O/${TAG:-r04}_pmc_gen.txt
cat $O/${TAG:-r04}_pmc_gen.txt
