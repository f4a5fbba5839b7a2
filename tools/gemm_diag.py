"""Timing decomposition of the gemm3 pair-mode kernel (SRNN_G3DIAG bits: 1 no MFMA, 8 no
epilogue) on the TBPTT shapes, interleaved in one process.  python tools/gemm_diag.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gemm_bench as GB  # noqa: E402

if __name__ == '__main__':
    bf, f32 = torch.bfloat16, torch.float32
    shapes = [
        (131072, 1024, 1024, False, True, bf, bf, 'mlp hidden fwd NT +bias'),
        (131072, 1024, 1024, False, False, bf, f32, 'mlp dgrad NN +mask'),
        (16384, 1024, 8192, False, True, bf, f32, 'mlp hidden NT K8192'),
    ]
    for rnd in range(2):
        for (M, N, K, tA, tB, dt, odt, tag) in shapes:
            for d in [int(v) for v in os.environ.get('DIAGS', '0,8').split(',')]:
                os.environ['SRNN_G3DIAG'] = str(d)
                GB.run(M, N, K, tA, tB, dt, odt, 5, '%s diag=%d' % (tag, d))
