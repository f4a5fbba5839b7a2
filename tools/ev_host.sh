set -e
mkdir -p gpurun_out
SRNN_GRAPH=0 timeout -k 10 200 python3 tools/host_prof.py 64 10 > gpurun_out/host_prof2.txt 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_persistent_errors.py tests/test_gpu_bench_parity.py tests/test_gpu_parity.py -m gpu -x -q -s --timeout 120 --timeout-method thread > gpurun_out/t_opt.log 2>&1
echo ok
