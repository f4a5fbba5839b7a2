set -e
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "bits" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05b4_tests.log 2>&1
tail -1 gpurun_out/r05b4_tests.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "bits" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05b4_tests2.log 2>&1
tail -1 gpurun_out/r05b4_tests2.log
TAG=r05b4 BS="512" bash tools/prof_step.sh
head -14 gpurun_out/r05b4_step_kernels_b512.txt
