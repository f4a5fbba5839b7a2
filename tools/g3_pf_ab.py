"""A/B of the gemm3p unit-1 fragment prefetch (SRNN_G3_PF) on the step's large GEMM shapes at
B = 512, interleaved in one process (rounds x variants)."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
import torch
import samplernn_hip as H

dev = 'cuda'
M = 512 * 1024


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


shapes = [('hid_fwd NT bf16', M, 1024, 1024, False, True, torch.bfloat16),
          ('da NN bf16', M, 1024, 1024, False, False, torch.bfloat16),
          ('up_fwd NT bf16', 32768, 16384, 1024, False, True, torch.bfloat16),
          ('dX NN fp32', 32768, 1024, 16384, False, False, torch.float32),
          ('out_fwd NT fp32', M, 256, 1024, False, True, torch.float32)]
res = {}
for rnd in range(3):
    for name, m, n, k, ta, tb, od in shapes:
        a = (torch.rand(k, m) * 2 - 1 if ta else torch.rand(m, k) * 2 - 1).to(dev, torch.bfloat16)
        b = (torch.rand(n, k) * 2 - 1 if tb else torch.rand(k, n) * 2 - 1).to(dev, torch.bfloat16)
        for pf in ('0', '1'):
            os.environ['SRNN_G3_PF'] = pf
            t = bench(lambda: H.gemm(a, b, transA=ta, transB=tb, out_dtype=od))
            res.setdefault((name, pf), []).append(t)
        del a, b
for name, *_ in shapes:
    r0, r1 = res[(name, '0')], res[(name, '1')]
    print('%-18s pf0 %s  pf1 %s  (min %.1f vs %.1f us)' % (name, ['%.1f' % x for x in r0],
                                                        ['%.1f' % x for x in r1], min(r0), min(r1)),
          flush=True)
