# GRU sweeps: early hand-off loads (MT > 1) + compile-time D forward; tests then bench A/B
bash tools/gsteps.sh \
 "300 python -u -m pytest tests/test_gpu_kernels.py -k 'gru_xcd' -v --timeout 120 --timeout-method thread > gpurun_out/r04i_tests.log 2>&1" \
 "240 python -u bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra > gpurun_out/r04i_b512.json 2> gpurun_out/r04i_b512.err" \
 "240 python -u bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra --batch 128 > gpurun_out/r04i_b128.json 2> gpurun_out/r04i_b128.err" \
 "300 TAG=r04i BS=512 bash tools/prof_step.sh"
