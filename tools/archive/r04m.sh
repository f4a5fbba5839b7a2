# padding-row hand-off loads skipped (B < 128) + side-stream bias sums: tests, bench 64 / 512
bash tools/gsteps.sh \
 "300 python -u -m pytest tests/test_gpu_kernels.py -k 'gru_xcd' -q -rf --timeout 120 --timeout-method thread > gpurun_out/r04m_tests.log 2>&1" \
 "240 python -u bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra --batch 64 > gpurun_out/r04m_b64.json 2> gpurun_out/r04m_b64.err" \
 "240 python -u bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra --batch 128 > gpurun_out/r04m_b128.json 2> gpurun_out/r04m_b128.err" \
 "240 python -u bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra > gpurun_out/r04m_b512.json 2> gpurun_out/r04m_b512.err" \
 "300 TAG=r04m BS=64 bash tools/prof_step.sh"
