"""Generation-tick skinny GEMMs in isolation: HIP-event time per launch (back-to-back
launches, weights cycled through NBUF copies so they are not L2-resident across launches,
as in the generation loop where the persistent sample loop runs in between) and, with
SRNN_SKINNY_DIAG=1, workgroup 0's stage timestamps.
  python tools/skinny_probe.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
import samplernn_hip as H  # noqa: E402

DEV = 'cuda'
NBUF = 4
for (M, N, K) in [(128, 19456, 1024), (128, 15360, 1024), (128, 16384, 1024)]:
    a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    ws = [torch.randn(N, K, device=DEV).to(torch.bfloat16) for _ in range(NBUF)]
    bias = torch.randn(N, device=DEV)
    out = torch.empty(M, N, device=DEV)
    ref = (a.float() @ ws[0].float().t()) + bias
    H.linear(a, ws[0], bias=bias, out=out)
    torch.cuda.synchronize()
    err = (out - ref).abs().max().item()
    for i in range(10):
        H.linear(a, ws[i % NBUF], bias=bias, out=out)
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 200
    e0.record()
    for i in range(n):
        H.linear(a, ws[i % NBUF], bias=bias, out=out)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000.0 / n
    gbs = N * K * 2 / (us * 1e-6) / 1e9
    print('%d x %d x %d: %.2f us/launch (weights %.1f GB/s), max err %.3g' % (M, N, K, us, gbs, err),
          flush=True)
    if os.environ.get('SRNN_SKINNY_DIAG') == '1':
        H.lib().dll.srnn_skinny_diag_dump()
