import os, sys
sys.path.insert(0, 'tools')
import torch
import gemm_bench as GB
bf = torch.bfloat16
for rnd in range(2):
    for (M, N, K) in ((131072, 1024, 1024), (131072, 1024, 256)):
        for tag in ('+mask', ''):
            for d in (0, 8):
                os.environ['SRNN_G3DIAG'] = str(d)
                GB.run(M, N, K, False, False, bf, bf, 5, 'NN %d %s diag=%d' % (K, tag or 'nomask', d))
