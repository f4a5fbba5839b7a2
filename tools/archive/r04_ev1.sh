# round-4 evidence, part 1: every GPU test, smoke, per-step kernel tables, generation timelines
bash tools/gsteps.sh \
 "700 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/r04_gpu_tests.log 2>&1" \
 "300 python3 -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r04_smoke.log 2>&1" \
 "400 TAG=r04 BS='512 128 64' bash tools/prof_step.sh"
