"""Time the persistent GRU forward (srnn_gru_seq_fwd) at B=128, D=1024, Fr=64 bf16."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
import samplernn_hip as H  # noqa: E402


def main():
    B, D, Fr = 128, 1024, 64
    T = torch.bfloat16
    g = torch.Generator(device='cuda').manual_seed(0)
    whh = (torch.randn(3 * D, D, device='cuda', generator=g) * 0.03).to(T)
    bhh = torch.randn(3 * D, device='cuda', generator=g) * 0.1
    gi = torch.randn(B * Fr, 3 * D, device='cuda', generator=g) * 0.5
    h0 = torch.zeros(B, D, device='cuda')
    h0T = h0.to(T)
    out = torch.empty(B, Fr, D, device='cuda')
    outT = torch.empty(B, Fr, D, device='cuda', dtype=T)
    gt = torch.empty(B, Fr, 4 * D, device='cuda')
    work = torch.zeros(4 * 64 + 1, device='cuda', dtype=torch.int32)

    def run():
        H.lib().call('srnn_gru_seq_fwd', H.BF16, B, D, Fr, H.ptr(gi), Fr * 3 * D, 3 * D,
                     H.ptr(h0), H.ptr(h0T), H.ptr(whh), H.ptr(bhh), H.ptr(out), H.ptr(outT),
                     Fr * D, D, H.ptr(gt), Fr * 4 * D, 4 * D, H.ptr(work), work.numel() * 4, H.stream())
    for _ in range(2):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        run()
    e1.record()
    e1.synchronize()
    print('gru_seq diag=%s: %.2f us/step, err=%d' % (os.environ.get('SRNN_GSEQ_DIAG', '0'),
          e0.elapsed_time(e1) * 1e3 / (5 * Fr), int(work[-1])))


if __name__ == '__main__':
    main()
