for m in 2 0 1 3 4; do
  for d in 0 8; do
    SRNN_G3MODE=$m SRNN_G3DIAG=$d timeout -k 10 60 python -c "
import sys,torch; sys.path.insert(0,'.'); import bench
dev=torch.device('cuda',0); torch.cuda.set_device(dev)
ms=[bench.kernel_roofline_gemm(dev,131072,1024,1024,torch.bfloat16,reps=20) for _ in range(3)]
print('mode $m diag $d', ' '.join('%.3f'%x for x in ms), 'ms  best %.0f TF/s'%(2*131072*1024*1024/min(ms)/1e9))
" || exit 1
  done
done
