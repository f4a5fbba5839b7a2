"""Times the generation loop's M = batch projections (srnn_gemm skinny path) in isolation:
bottom-tier upsampling 128 x 16384 x 1024 and top-tier 128 x 4096 x 1024 (bf16 -> fp32).
  python tools/skinny_bench.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
import samplernn_hip as H  # noqa: E402

DEV = 'cuda'
for (M, N, K) in [(128, 16384, 1024), (128, 4096, 1024), (128, 3072, 1024)]:
    a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = torch.randn(N, K, device=DEV).to(torch.bfloat16)
    bias = torch.randn(N, device=DEV)
    out = torch.empty(M, N, device=DEV)
    for _ in range(5):
        H.linear(a, w, bias=bias, out=out)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        H.linear(a, w, bias=bias, out=out)
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) / 50 * 1e3
    print('skinny %dx%dx%d: %.1f us (%.2f TB/s of weights)' % (M, N, K, us, N * K * 2 / us / 1e6),
          flush=True)
