#!/bin/bash
# Round evidence in one GPU call, summaries only (the raw rocpd databases stay on the box):
#   bash tools/round_evidence.sh r02
# -> gpurun_out/<tag>_bench.json, <tag>_kernel_stats.csv (kernel trace of the same bench command),
#    <tag>_pmc_gemm.txt (FETCH/WRITE passes over the roofline GEMM), <tag>_pmc_gen.txt
#    (FETCH/WRITE passes over the generation loop, tools/pmc_gen.py), <tag>_mfma.txt
set -e
tag=${1:-r02}
R=$PWD
O=$R/gpurun_out
S=/tmp/ev_$tag
mkdir -p $O $S
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py > $O/${tag}_bench.json 2> $O/${tag}_bench.err
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $S/prof -o run -- python3 $R/bench.py > $O/${tag}_prof.log 2>&1
python3 $R/tools/rocpd_summary.py stats $(find $S/prof -name '*.db' | head -1) > $O/${tag}_kernel_stats.csv
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $S/gf -o run -- python3 $R/tools/roofline_kernel.py gemm > $O/${tag}_pmc_gf.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $S/gw -o run -- python3 $R/tools/roofline_kernel.py gemm > $O/${tag}_pmc_gw.log 2>&1
{
  echo "# rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, python tools/roofline_kernel.py gemm"
  echo "# (bench.py roofline kernel: 131072x1024x1024 bf16 bias+relu, gemm3p_kernel). FETCH_SIZE is kB and must be x2 on gfx950 (MI355X_MICROARCH.md HBM section)."
  python3 $R/tools/rocpd_summary.py pmc $(find $S/gf -name '*.db' | head -1) gemm3
  python3 $R/tools/rocpd_summary.py pmc $(find $S/gw -name '*.db' | head -1) gemm3
} > $O/${tag}_pmc_gemm.txt
gen="python3 $R/tools/gen_prof.py 128 20"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $S/nf -o run -- $gen > $O/${tag}_pmc_nf.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $S/nw -o run -- $gen > $O/${tag}_pmc_nw.log 2>&1
python3 $R/tools/pmc_gen.py $(find $S/nf -name '*.db' | head -1) $(find $S/nw -name '*.db' | head -1) > $O/${tag}_pmc_gen.txt
rm -rf $S
echo done
