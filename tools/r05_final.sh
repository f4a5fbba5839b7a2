#!/bin/bash
# Round-5 evidence at HEAD: bench (default args) + smoke, the dTab and da1 sites' and the four
# generation lines' PMC passes, the per-step kernel tables at B = 512 / 64.
set -e
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05f}
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
TAG=$TAG SITE=dtab_scatter ROWS=512 KERNELS="dtab_prep_kernel dtab_pk_kernel" bash tools/pmc_site.sh > /dev/null
# the da1 GEMM (the grouped-bits + max |C| instantiation; template name without spaces)
TAG=$TAG SITE=mlp_da1_gemm ROWS=512 KERNELS="gemm3p_kernel<__hip_bfloat16,true,true,true,2,true,true,0>" bash tools/pmc_site.sh > /dev/null
for k in gen gen_fp32 gen_e gen_e_fp32; do TAG=$TAG KIND=$k bash tools/pmc_gen.sh > /dev/null; done
TAG=$TAG BS="512 64" bash tools/prof_step.sh
echo done
