set -e
TAG=r05g2 bash tools/r05_gen.sh
SRNN_GEN_DIAG=20 timeout -k 10 120 python3 tools/gen_diag.py bf16 > gpurun_out/r05g2_diag.txt 2>&1
grep -h "gen" gpurun_out/r05g2_bench.err | head -20
