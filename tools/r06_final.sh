#!/bin/bash
# Round-6 evidence at the final sources (one pass): the GPU suite, smoke, the default bench line,
# the dTab and da1 sites' and the four generation lines' PMC passes (bench.py reads their
# traffic when the csrc hash matches), per-step kernel tables at B = 512 / 64 and the
# generation kernel timelines.  Each GPU step under its own time limit; any failure ends it.
set -e
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r06z}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
TAG=$TAG SITE=dtab_scatter ROWS=512 KERNELS="dtab_prep_kernel dtab_pk_kernel" bash tools/pmc_site.sh > /dev/null
TAG=$TAG SITE=mlp_da1_gemm ROWS=512 KERNELS="gemm3p_kernel<__hip_bfloat16,true,true,true,2,true,true,0,0>" bash tools/pmc_site.sh > /dev/null
for k in gen gen_fp32 gen_e gen_e_fp32; do TAG=$TAG KIND=$k bash tools/pmc_gen.sh > /dev/null; done
TAG=$TAG BS="512 64" bash tools/prof_step.sh
TAG=$TAG DTS="bf16 fp32" bash tools/prof_gen.sh
echo done
