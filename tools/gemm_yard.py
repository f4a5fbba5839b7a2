"""Yardstick: hipBLASLt (torch.matmul, bf16 in / bf16 or fp32 out) vs the HIP gemm3 path
(samplernn_hip.gemm) on the TBPTT step's large GEMM shapes at B = 512."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
import torch
import samplernn_hip as H

dev = 'cuda'
M = 512 * 1024


def bench(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


shapes = [('hid_fwd NT', M, 1024, 1024, False, True),
          ('da NN', M, 1024, 1024, False, False),
          ('dW TN', 1024, 1024, M, True, False),
          ('out_fwd NT', M, 256, 1024, False, True),
          ('up_fwd NT', 32768, 16384, 1024, False, True),
          ('dWup TN', 1024, 16384, 32768, True, False)]
for name, m, n, k, ta, tb in shapes:
    a = (torch.randn(k, m) if ta else torch.randn(m, k)).to(dev, torch.bfloat16)
    b = (torch.randn(n, k) if tb else torch.randn(k, n)).to(dev, torch.bfloat16)
    fl = 2.0 * m * n * k
    for od in (torch.bfloat16, torch.float32):
        def ours():
            H.gemm(a, b, transA=ta, transB=tb, out_dtype=od)
        A = a.t() if ta else a
        B = b.t() if tb else b
        if od == torch.bfloat16:
            def lt():
                torch.matmul(A, B)
        else:
            def lt():
                torch.matmul(A, B, out_dtype=torch.float32) if hasattr(torch, 'mm') else None
        try:
            t_o = bench(ours)
        except Exception as e:  # noqa: BLE001
            t_o = float('nan')
            print('ours failed', e)
        try:
            t_l = bench(lt)
        except Exception as e:  # noqa: BLE001
            t_l = float('nan')
        print('%-12s %6dx%6dx%6d out %-8s ours %8.1f us (%6.1f TF/s)  hipblaslt %8.1f us (%6.1f TF/s)'
              % (name, m, n, k, str(od)[6:], t_o, fl / t_o / 1e6, t_l, fl / t_l / 1e6), flush=True)
