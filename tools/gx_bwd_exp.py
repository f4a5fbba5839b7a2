"""Timing experiment on the packed reverse GRU sweep (gru_xcd_bwd_pk_kernel): per-step time
with SRNN_GX_EXP = 0 (normal), 64 (no operand fetch for the next step), 1 (no output stores),
65 (neither) -- results are invalid in the experiment modes; only the time is read.  B rows
(512 and 64: configs[3] at N = 1 and N = 8), D = 1024, 64 frames, interleaved rounds."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
import samplernn_hip as H  # noqa: E402

dev = 'cuda'
D, Fr = 1024, 64
T = torch.bfloat16
for B in (512, 64):
    g = torch.Generator(device=dev).manual_seed(3)
    whh = (torch.randn(3 * D, D, device=dev, generator=g) * 0.03).to(T)
    whh_t = whh.t().contiguous()
    h0 = torch.zeros(B, D, device=dev)
    out = torch.randn(B, Fr, D, device=dev, generator=g) * 0.5
    gt = torch.rand(B, Fr, 4 * D, device=dev, generator=g)
    nb = H.gru_xcd_bwd_work_bytes(T, B, D)
    wb = torch.empty(nb, device=dev, dtype=torch.uint8)
    dy = torch.randn(B, Fr, D, device=dev, generator=g) * 0.1
    dgh = torch.empty(B, Fr, 3 * D, device=dev, dtype=T)
    dgi = torch.empty(B, Fr, 3 * D, device=dev, dtype=T)
    bsum = torch.empty(B, 4 * D, device=dev)
    ddir0 = torch.empty(B, D, device=dev)

    def bwd():
        H.lib().call('srnn_gru_xcd_bwd2', H.BF16, B, D, Fr, H.ptr(dy), Fr * D, D, H.ptr(gt),
                     Fr * 4 * D, 4 * D, H.ptr(out), Fr * D, D, H.ptr(h0), H.ptr(whh_t), None,
                     H.ptr(dgh), None, H.ptr(dgi), H.ptr(bsum), Fr * 3 * D, 3 * D, H.ptr(ddir0),
                     H.ptr(wb), nb, H.stream())
    res = {}
    for rnd in range(4):
        for mode in ('0', '64', '1', '65'):
            os.environ['SRNN_GX_EXP'] = mode
            bwd()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                bwd()
            e1.record()
            e1.synchronize()
            res.setdefault(mode, []).append(e0.elapsed_time(e1) / 5 * 1e3 / Fr)
    os.environ['SRNN_GX_EXP'] = '0'
    H.check_persistent_errors()
    print('B=%d: ' % B + '  '.join('exp %s: %.2f us/step (min of %d)' % (m, min(v), len(v))
                                   for m, v in res.items()), flush=True)
