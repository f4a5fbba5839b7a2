#!/bin/bash
# PMC passes over tools/dtab_bench.py (the dTab scatter), one counter group per run
set -e
out=${1:-gpurun_out/pmc_dtab}
R=$PWD
mkdir -p $out
export TMPDIR=/tmp
cmd="python3 $R/tools/dtab_bench.py"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $R/$out/p1 -o run -- $cmd > $R/$out/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $R/$out/p2 -o run -- $cmd > $R/$out/p2.log 2>&1
echo done
