set -e
TAG=r05 BS="64 512" bash tools/prof_step.sh
for k in gen gen_fp32 gen_e gen_e_fp32; do TAG=r05 KIND=$k bash tools/pmc_gen.sh > /dev/null; done
ls gpurun_out/r05_pmc_*
