"""Time srnn_mlp_dtab at the TBPTT shape (B=128 rows x T=1024, D=1024, FS0=16, Q=256)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
import samplernn_hip as H  # noqa: E402


def main():
    B, T, D, FS0, Q = 128, 1024, 1024, 16, 256
    dt = torch.bfloat16 if os.environ.get('DT', 'bf16') == 'bf16' else torch.float32
    g = torch.Generator(device='cuda').manual_seed(0)
    x = torch.randint(0, Q, (B, T + FS0 - 1), device='cuda', generator=g)
    da = (torch.randn(B * T, D, device='cuda', generator=g) * 1e-4).to(dt)
    out = torch.empty(Q, FS0 * D, device='cuda', dtype=torch.bfloat16)
    work = torch.empty(Q * FS0 * D, device='cuda', dtype=torch.int64)

    def run():
        H.lib().call('srnn_mlp_dtab', H.dcode(dt), H.ptr(da), D, H.ptr(x), x.shape[1], 0, B, T,
                     H.ptr(out), H.BF16, D, FS0, Q, H.ptr(work), work.numel() * 8, H.stream())
    for _ in range(3):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        run()
    e1.record()
    e1.synchronize()
    print('dtab %s: %.3f ms' % (dt, e0.elapsed_time(e1) / 10))


if __name__ == '__main__':
    main()
