"""Phase timestamps of the XCD-grouped GRU forward sweep (SRNN_GRU_DIAG=1: workgroup 0,
thread 0 stamps s_memrealtime after the poll, the MMA + reduction write, the barrier, the
gate math + publish and the output stores of every (step, tile)); B = 512 (4 tiles per group)
and B = 128, D = 1024, 64 frames, bf16.
  SRNN_GRU_DIAG=1 python tools/archive/gru_stamp_probe.py [B]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
import samplernn_hip as H  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
D, Fr, T = 1024, 64, torch.bfloat16
dev = 'cuda'
g = torch.Generator(device=dev).manual_seed(0)
whh = (torch.randn(3 * D, D, device=dev, generator=g) * 0.03).to(T)
bhh = torch.randn(3 * D, device=dev, generator=g) * 0.1
gi = torch.randn(B, Fr, 3 * D, device=dev, generator=g) * 0.5
h0 = torch.randn(B, D, device=dev, generator=g) * 0.5
nf = H.gru_xcd_work_bytes(T, B, D)
out = torch.empty((B, Fr, D), device=dev)
outT = torch.empty((B, Fr, D), device=dev, dtype=T)
gt = torch.empty((B, Fr, 4 * D), device=dev)
hp = torch.empty((B, Fr, D), device=dev, dtype=T)
for it in range(3):
    wf = torch.zeros(nf, device=dev, dtype=torch.uint8)
    H.lib().call('srnn_gru_xcd_fwd2', H.BF16, B, D, Fr, H.ptr(gi), Fr * 3 * D, 3 * D, H.ptr(h0),
                 H.ptr(whh), H.ptr(bhh), H.ptr(out), H.ptr(outT), Fr * D, D, H.ptr(gt),
                 Fr * 4 * D, 4 * D, H.ptr(hp), H.ptr(wf), nf, H.stream())
    torch.cuda.synchronize()
H.lib().dll.srnn_gru_diag_dump()
