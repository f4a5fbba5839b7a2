"""Per-step time of the GRU cell kernels at the TBPTT shape (B=128, D=1024, bf16): a chain
of dependent steps as in the tier forward (gi precomputed), events around N steps."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
import samplernn_hip as H  # noqa: E402


def main():
    B, D, N = 128, 1024, 64
    T = torch.bfloat16
    g = torch.Generator(device='cuda').manual_seed(0)
    whh = (torch.randn(3 * D, D, device='cuda', generator=g) * 0.03).to(T)
    bhh = torch.randn(3 * D, device='cuda', generator=g) * 0.1
    gi = torch.randn(N, B, 3 * D, device='cuda', generator=g) * 0.5
    hf = torch.zeros(N + 1, B, D, device='cuda')
    hl = torch.zeros(N + 1, B, D, device='cuda', dtype=T)
    gates = torch.empty(N, B, 4 * D, device='cuda')

    def fwd():
        for t in range(N):
            H.lib().call('srnn_gru_cell', H.BF16, B, D, D, None, D, None, None, H.ptr(gi[t]), 3 * D,
                         H.ptr(hl[t]), D, H.ptr(hf[t]), D, H.ptr(whh), H.ptr(bhh), H.ptr(hf[t + 1]),
                         D, H.ptr(hl[t + 1]), D, H.ptr(gates[t]), 4 * D, H.stream())
    for _ in range(3):
        fwd()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        fwd()
    e1.record()
    e1.synchronize()
    print('gru_cell fwd: %.2f us/step (wall incl. launch gaps)' % (e0.elapsed_time(e1) * 1e3 / (5 * N)))


if __name__ == '__main__':
    main()
