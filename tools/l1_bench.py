"""Times the bf16 training L1 gather (srnn_mlp_l1) at config-B shape, LDS-resident table vs the
L2-gather kernel (SRNN_L1_LDS), HIP events; also usable under rocprofv3 --pmc.
  python tools/l1_bench.py [modes=1,0] [reps=20]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
import samplernn_hip as H  # noqa: E402

DEV = 'cuda'
B, Tl, D, FS0, Q = 128, 1024, 1024, 16, 256
modes = (sys.argv[1] if len(sys.argv) > 1 else '1,0').split(',')
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
g = torch.Generator().manual_seed(1)
tab = (torch.randn(FS0, Q, D, generator=g) * 0.1).to(DEV, torch.bfloat16)
x = torch.randint(0, Q, (B, Tl + FS0 - 1), generator=g).to(DEV)
up = torch.randn(B * Tl, D, generator=g).to(DEV, torch.bfloat16)
out = torch.empty(B * Tl, D, device=DEV, dtype=torch.bfloat16)


def run():
    H.lib().call('srnn_mlp_l1', H.BF16, H.ptr(tab), H.ptr(x), x.shape[1], 0, B, Tl, H.BF16,
                 H.ptr(up), D, H.ptr(out), D, D, FS0, Q, H.stream())


for rnd in range(2):
    for m in modes:
        os.environ['SRNN_L1_LDS'] = m
        for _ in range(3):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        print('mode %s: %.1f us  (%.2f TB/s of upper+out)' % (m, us, 2 * up.numel() * 2 / us / 1e6),
              flush=True)
