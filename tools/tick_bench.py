"""Times the generation tick's products in isolation (B = 128, D = 1024, bf16): the GRU cell
with its input projection (srnn_gru_cell, x given) and the tier upsampling (128 x 16384 x 1024,
bf16 -> fp32), 50 back-to-back launches each between HIP events.
  python tools/tick_bench.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
import samplernn_hip as H  # noqa: E402

DEV = 'cuda'


def timed(fn, n=50):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    B, D = 128, 1024
    T = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(0)
    x = torch.randn(B, D, device=DEV, generator=g).to(T)
    h = torch.randn(B, D, device=DEV, generator=g).to(T)
    hf = h.float()
    wih = (torch.randn(3 * D, D, device=DEV, generator=g) * 0.03).to(T)
    whh = (torch.randn(3 * D, D, device=DEV, generator=g) * 0.03).to(T)
    bih = torch.zeros(3 * D, device=DEV)
    bhh = torch.zeros(3 * D, device=DEV)
    hout = torch.empty(B, D, device=DEV)
    hlp = torch.empty(B, D, device=DEV, dtype=T)

    def cell():
        H.lib().call('srnn_gru_cell', H.BF16, B, D, D, H.ptr(x), D, H.ptr(wih), H.ptr(bih), None, 0,
                     H.ptr(h), D, H.ptr(hf), D, H.ptr(whh), H.ptr(bhh), H.ptr(hout), D, H.ptr(hlp),
                     D, None, 0, H.stream())
    us = timed(cell)
    wbytes = 2 * 3 * D * D * 2
    print('gru_cell B=%d D=%d (x given): %.2f us (%.2f TB/s of weights)'
          % (B, D, us, wbytes / us / 1e6), flush=True)
    for (M, N, K) in [(128, 16384, 1024), (128, 4096, 1024)]:
        a = torch.randn(M, K, device=DEV, generator=g).to(T)
        w = torch.randn(N, K, device=DEV, generator=g).to(T)
        bias = torch.randn(N, device=DEV, generator=g)
        out = torch.empty(M, N, device=DEV)
        us = timed(lambda: H.linear(a, w, bias=bias, out=out))
        print('upsampling %dx%dx%d: %.2f us (%.2f TB/s of weights)' % (M, N, K, us, N * K * 2 / us / 1e6),
              flush=True)


if __name__ == '__main__':
    main()
