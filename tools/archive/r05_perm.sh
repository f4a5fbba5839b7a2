set -e
# dTab scatter A/B: lib_A (before), lib_B (row-major + v_perm), lib_C (+ unrolled prefetch ring)
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "dtab" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05pm_tests.log 2>&1
tail -1 gpurun_out/r05pm_tests.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_parity.py tests/test_gpu_parity_big.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05pm_tests2.log 2>&1
tail -1 gpurun_out/r05pm_tests2.log
TAG=${TAG:-r05pm} ROUNDS=${ROUNDS:-3} BS="${BS:-512 64}" bash tools/r05_soab.sh
