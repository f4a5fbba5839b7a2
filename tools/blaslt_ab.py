"""gemm3 (H.gemm) against the ROCm BLAS behind torch.mm (hipBLASLt) on the TBPTT step's large
plain GEMM shapes at B = 512 (bf16 operands), interleaved in one process.  torch.mm returns
bf16; out_dtype=fp32 where this torch offers it."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..',
                                'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
import samplernn_hip as H  # noqa: E402


def bench(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


M = 512 * 1024
shapes = [('hid_fwd NT', M, 1024, 1024, False, True, torch.bfloat16),
          ('dW_hid TN', 1024, 1024, M, True, False, torch.float32),
          ('up_fwd NT', 32768, 16384, 1024, False, True, torch.bfloat16),
          ('up_dX NN', 32768, 1024, 16384, False, False, torch.float32),
          ('up_dW TN', 16384, 1024, 32768, True, False, torch.float32),
          ('out_fwd NT', M, 256, 1024, False, True, torch.float32),
          ('dW_ih TN', 3072, 1024, 32768, True, False, torch.float32),
          ('dW_out TN', 256, 1024, M, True, False, torch.float32),
          ('gi_fwd NT', 32768, 3072, 1024, False, True, torch.float32),
          ('dX_ih NN', 32768, 1024, 3072, False, False, torch.float32)]
try:
    torch.mm(torch.ones(16, 16, device='cuda', dtype=torch.bfloat16),
             torch.ones(16, 16, device='cuda', dtype=torch.bfloat16), out_dtype=torch.float32)
    has_od = True
except Exception as e:  # noqa: BLE001
    print('torch.mm out_dtype unavailable: %s' % e)
    has_od = False
res = {}
for rnd in range(3):
    for name, m, n, k, ta, tb, od in shapes:
        a = (torch.rand(k, m) * 2 - 1 if ta else torch.rand(m, k) * 2 - 1).to('cuda', torch.bfloat16)
        b = (torch.rand(n, k) * 2 - 1 if tb else torch.rand(k, n) * 2 - 1).to('cuda', torch.bfloat16)
        A = a.t() if ta else a
        Bm = b.t() if tb else b
        res.setdefault((name, 'gemm3'), []).append(
            bench(lambda: H.gemm(a, b, transA=ta, transB=tb, out_dtype=od)))
        res.setdefault((name, 'torch bf16'), []).append(bench(lambda: torch.mm(A, Bm)))
        if has_od and od == torch.float32:
            res.setdefault((name, 'torch fp32'), []).append(
                bench(lambda: torch.mm(A, Bm, out_dtype=torch.float32)))
        del a, b, A, Bm
for name, m, n, k, *_ in shapes:
    line = '%-12s %6dx%5dx%6d' % (name, m, n, k)
    for v in ('gemm3', 'torch bf16', 'torch fp32'):
        r = res.get((name, v))
        if r:
            line += '  %s %.1f us (%.0f TF/s)' % (v, min(r), 2.0 * m * n * k / min(r) / 1e6)
    print(line, flush=True)
