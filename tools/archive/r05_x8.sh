set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "dtab" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05x8_tests.log 2>&1
tail -1 gpurun_out/r05x8_tests.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_parity.py tests/test_gpu_parity_big.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05x8_tests2.log 2>&1
tail -1 gpurun_out/r05x8_tests2.log
TAG=r05x8 VAR=SRNN_DTAB_X8 BS="512 64" bash tools/r05_envab.sh
