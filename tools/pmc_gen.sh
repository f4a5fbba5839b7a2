#!/bin/bash
# HBM traffic of a generation line, two separate rocprofv3 --pmc passes:
#   TAG=r05 KIND=gen bash tools/pmc_gen.sh      (KIND: gen | gen_fp32 | gen_e | gen_e_fp32)
#   ->  gpurun_out/<TAG>_pmc_<KIND>.txt (copy to profiles/; bench.py reads r*_pmc_<KIND>.txt)
set -e
R=$PWD; O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
KIND=${KIND:-gen}
case $KIND in
  gen) args="bf16 20" ;;
  gen_fp32) args="fp32 12" ;;
  gen_e) args="bf16 6 e" ;;
  gen_e_fp32) args="fp32 4 e" ;;
esac
cmd="python3 $R/tools/gen_prof.py $args"
rm -rf /tmp/gf_$KIND /tmp/gw_$KIND
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d /tmp/gf_$KIND -o run -- $cmd > $O/pmc_${KIND}_f.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d /tmp/gw_$KIND -o run -- $cmd > $O/pmc_${KIND}_w.log 2>&1
python3 $R/tools/pmc_gen.py $(find /tmp/gf_$KIND -name '*.db' | head -1) $(find /tmp/gw_$KIND -name '*.db' | head -1) "$KIND: tools/gen_prof.py $args" > $O/${TAG:-r05}_pmc_$KIND.txt
cat $O/${TAG:-r05}_pmc_$KIND.txt
