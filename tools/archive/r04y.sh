# two-rank gloo rehearsal of bench.py at N = 2 on one GPU, with the extra lines (weak_64,
# weak_512): exercises the N > 1 code paths the driver's scaling run takes (not a number)
SRNN_DIST_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 2 --no-gen --no-cpu \
  > gpurun_out/r04_dp2_rehearsal.json 2> gpurun_out/r04_dp2_rehearsal.err
