#!/bin/bash
# HBM traffic of one bench.py launch site per step, two separate rocprofv3 --pmc passes:
#   SITE=dtab_scatter ROWS=512 KERNELS="dtab_prep_kernel dtab_pk_kernel" bash tools/pmc_site.sh
# -> gpurun_out/<TAG>_pmc_<site>_b<rows>.txt (copy to profiles/ for bench.py's roofline.traffic)
set -e
R=$PWD; O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
rm -rf /tmp/pf /tmp/pw                                  # (a previous site's databases)
cmd="python3 $R/bench.py --steps 3 --warmup 2 --no-gen --no-cpu --no-extra --batch $ROWS"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d /tmp/pf -o run -- $cmd > $O/pmc_${SITE}_f.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d /tmp/pw -o run -- $cmd > $O/pmc_${SITE}_w.log 2>&1
python3 $R/tools/pmc_site.py $SITE $ROWS $(find /tmp/pf -name '*.db' | head -1) $(find /tmp/pw -name '*.db' | head -1) $KERNELS > $O/${TAG:-r04}_pmc_${SITE}_b${ROWS}.txt
cat $O/${TAG:-r04}_pmc_${SITE}_b${ROWS}.txt
