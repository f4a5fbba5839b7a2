"""Times a few small-grid TBPTT GEMM shapes on each path (HIP events): auto dispatch vs the
256-tile kernel forced (tile 5), and the batched dWp = dTab^T E against its single-GEMM form.
  python tools/gemm_shapes.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
import samplernn_hip as H  # noqa: E402

DEV = 'cuda'


def timeit(fn, reps=50):
    for _ in range(10):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    bf = torch.bfloat16
    for (M, N, K) in ((2048, 3072, 1024), (2048, 4096, 1024), (2048, 1024, 3072),
                      (2048, 1024, 4096)):
        A = torch.randn(M, K, device=DEV).to(bf)
        W = torch.randn(N, K, device=DEV).to(bf)
        b = torch.randn(N, device=DEV)
        out = torch.empty(M, N, device=DEV)
        for tile in (-1, 5):
            us = timeit(lambda: H.gemm(A, W, transB=True, out=out, bias=b, tile=tile))
            print('NT+bias %5d x %5d x %5d tile=%2d %8.1f us %7.1f TF/s' %
                  (M, N, K, tile, us, 2.0 * M * N * K / us / 1e6), flush=True)
    Q, FS0, D = 256, 16, 1024
    dtabT = torch.randn(Q, FS0 * D, device=DEV).to(bf)
    ET = torch.randn(Q, Q, device=DEV).to(bf)
    dWp = torch.empty(FS0, D, Q, device=DEV)
    us = timeit(lambda: H.gemm(dtabT, ET, transA=True, out=dWp, M=D, N=Q, K=Q, lda=FS0 * D,
                               ldb=Q, ldc=Q, batch=FS0, sA=D, sB=0, sC=D * Q))
    print('dWp batched             %8.1f us' % us, flush=True)
    ref = dWp.clone()
    for tile in (-1, 5):
        us = timeit(lambda: H.gemm(dtabT, ET, transA=True, out=dWp, M=FS0 * D, N=Q, K=Q,
                                   lda=FS0 * D, ldb=Q, ldc=Q, tile=tile))
        err = (dWp - ref).abs().max().item()
        print('dWp single tile=%2d      %8.1f us  max diff vs batched %.3g' % (tile, us, err),
              flush=True)


if __name__ == '__main__':
    main()
