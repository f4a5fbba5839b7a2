# round-4 evidence, part 2: PMC passes at this csrc hash, then the bench (reads them from profiles/)
bash tools/gsteps.sh \
 "200 SITE=dtab_scatter ROWS=512 KERNELS='dtab_prep_kernel dtab_pk_kernel dtab_pos_kernel' TAG=r04 bash tools/pmc_site.sh" \
 "200 TAG=r04 bash tools/pmc_gen.sh" \
 "10 cp gpurun_out/r04_pmc_dtab_scatter_b512.txt gpurun_out/r04_pmc_gen.txt profiles/" \
 "300 TAG=r04 DTS='bf16 fp32' bash tools/prof_gen.sh" \
 "600 python3 bench.py > gpurun_out/r04_bench.json 2> gpurun_out/r04_bench.err"
