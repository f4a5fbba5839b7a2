"""Phase timestamps of the XCD-grouped GRU forward (SRNN_GRU_DIAG=1): B=128, D=1024, Fr=64."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
import samplernn_hip as H  # noqa: E402

B, D, Fr = int(sys.argv[1]) if len(sys.argv) > 1 else 128, 1024, 64
dev = 'cuda'
T = torch.bfloat16
whh = (torch.randn(3 * D, D) * 0.03).to(dev, T)
bhh = torch.zeros(3 * D, device=dev)
gi = torch.randn(B * Fr, 3 * D, device=dev) * 0.5
h0 = torch.zeros(B, D, device=dev)
out = torch.empty(B, Fr, D, device=dev)
outT = torch.empty(B, Fr, D, device=dev, dtype=T)
gt = torch.empty(B, Fr, 4 * D, device=dev)
nb = H.gru_xcd_work_bytes(T, B, D)
work = torch.empty(nb, device=dev, dtype=torch.uint8)
for _ in range(3):
    H.lib().call('srnn_gru_xcd_fwd', H.BF16, B, D, Fr, H.ptr(gi), Fr * 3 * D, 3 * D, H.ptr(h0),
                 H.ptr(whh), H.ptr(bhh), H.ptr(out), H.ptr(outT), Fr * D, D, H.ptr(gt),
                 Fr * 4 * D, 4 * D, H.ptr(work), nb, H.stream())
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
H.lib().call('srnn_gru_xcd_fwd', H.BF16, B, D, Fr, H.ptr(gi), Fr * 3 * D, 3 * D, H.ptr(h0),
             H.ptr(whh), H.ptr(bhh), H.ptr(out), H.ptr(outT), Fr * D, D, H.ptr(gt),
             Fr * 4 * D, 4 * D, H.ptr(work), nb, H.stream())
e1.record()
e1.synchronize()
print('gru_xcd fwd %.1f us (%.2f us/step)' % (e0.elapsed_time(e1) * 1e3, e0.elapsed_time(e1) * 1e3 / Fr))
H.lib().dll.srnn_gru_diag_dump()
