"""Split-K weight-gradient shapes of the TBPTT step: ordered partial sums
(SRNN_G3_SPLITK_PART=1, default) vs fp32 atomics into a zeroed C (=0), interleaved in one
process, plus a check against torch.mm.  python tools/gemm_splitk.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gemm_bench as GB  # noqa: E402

H = GB.H
DEV = 'cuda'

if __name__ == '__main__':
    bf = torch.bfloat16
    shapes = [(256, 1024, 131072, 'mlp out wgrad TN'), (1024, 1024, 131072, 'mlp wgrad TN'),
              (3072, 1024, 8192, 'gru wgrad TN'), (16384, 1024, 8192, 'upsample wgrad TN'),
              (4096, 1024, 2048, 'top upsample wgrad TN'), (3072, 1024, 2048, 'top gru wgrad TN')]
    for rnd in range(2):
        for M, N, K, tag in shapes:
            A = torch.randn(K, M, device=DEV).to(bf)
            B = torch.randn(K, N, device=DEV).to(bf)
            ref = torch.mm(A.t().float(), B.float())
            for v in ('1', '0'):
                os.environ['SRNN_G3_SPLITK_PART'] = v
                out = torch.empty(M, N, device=DEV)
                ms = GB.timeit(lambda: H.gemm(A, B, transA=True, out=out))
                err = ((out - ref).abs().max() / ref.abs().max()).item()
                print('%-24s part=%s %7.3f ms %7.1f TFLOP/s  rel err %.2e' % (
                    tag, v, ms, 2.0 * M * N * K / ms / 1e9, err), flush=True)
