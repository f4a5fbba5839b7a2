"""Row-pitch experiment: gemm3 on the TBPTT shapes with the output (and operand) row pitch
padded past the power of two (L2 channel spread of the epilogue stores).
python tools/gemm_pad.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gemm_bench as GB  # noqa: E402

H = GB.H
DEV = 'cuda'


def run(M, N, K, tB, dt, odt, pad_c, pad_a, tag, mask=False, bias=False):
    A = torch.randn(M, K + pad_a, device=DEV).to(dt)[:, :K]
    B = torch.randn(N, K, device=DEV).to(dt) if tB else torch.randn(K, N, device=DEV).to(dt)
    out = torch.empty(M, N + pad_c, device=DEV, dtype=odt)[:, :N]
    kw = {}
    if mask:
        kw['mask'] = torch.randn(M, N + pad_c, device=DEV).to(dt)[:, :N]
    if bias:
        kw['bias'] = torch.randn(N, device=DEV)
        kw['relu'] = True
    ms = GB.timeit(lambda: H.gemm(A, B, transB=tB, out=out, tile=5, **kw))
    print('%-28s padC=%3d padA=%3d %7.3f ms %8.1f TFLOP/s' % (tag, pad_c, pad_a, ms,
                                                           2.0 * M * N * K / ms / 1e9), flush=True)


if __name__ == '__main__':
    bf, f32 = torch.bfloat16, torch.float32
    for rnd in range(2):
        for pc, pa in ((0, 0), (64, 0), (128, 0), (256, 0), (64, 64), (0, 64)):
            run(131072, 1024, 1024, True, bf, bf, pc, pa, 'hidden fwd NT +bias', bias=True)
            run(131072, 1024, 1024, False, bf, f32, pc, pa, 'dgrad NN +mask', mask=True)
