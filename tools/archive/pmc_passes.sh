#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, MI355X_MICROARCH.md PMC slots) for the
# generation sample loop (HBM bytes) and the TBPTT step (MFMA busy of the GRU / GEMM kernels).
# Run on the GPU box from the repo root:  bash tools/pmc_passes.sh gpurun_out/pmc
set -e
out=${1:-gpurun_out/pmc}
R=$PWD
mkdir -p $out
export TMPDIR=/tmp
gen="python3 $R/tools/gen_prof.py bf16 8"
tb="python3 $R/bench.py --steps 2 --warmup 1 --no-gen --no-cpu"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $R/$out/gen_fetch -o run -- $gen > $R/$out/gen_fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $R/$out/gen_write -o run -- $gen > $R/$out/gen_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES -d $R/$out/tb_mfma -o run -- $tb > $R/$out/tb_mfma.log 2>&1
echo done
