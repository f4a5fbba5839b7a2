#!/bin/bash
# Round evidence in one GPU call (run from the repo root on the GPU box):
#   bash tools/profile_round.sh r02
# -> gpurun_out/<tag>_bench.json (bench.py default run), gpurun_out/<tag>_prof/ (kernel trace of
#    the same command), gpurun_out/<tag>_pmc_{fetch,write}/ (PMC passes over the roofline kernel)
set -e
tag=${1:-r02}
R=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${tag}_prof -o run -- python3 $R/bench.py > $R/gpurun_out/${tag}_prof.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/${tag}_pmc_fetch -o run -- python3 $R/tools/roofline_kernel.py gemm > $R/gpurun_out/${tag}_pmc_fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/${tag}_pmc_write -o run -- python3 $R/tools/roofline_kernel.py gemm > $R/gpurun_out/${tag}_pmc_write.log 2>&1
echo done
