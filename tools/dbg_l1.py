"""debug: LDS gather kernel vs reference on one small case (prints error pattern)."""
import os, sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
import samplernn_hip as H
DEV = 'cuda'
B, Tl, D, FS0, Q = 8, 1024, 256, 16, 256
g = torch.Generator().manual_seed(1)
tab = torch.randn(FS0, Q, D, generator=g).to(DEV, torch.bfloat16)
x = torch.randint(0, Q, (B, Tl + FS0 - 1), generator=g).to(DEV)
up = torch.randn(B * Tl, D, generator=g).to(DEV, torch.bfloat16)
for mode in sys.argv[1:] or ['0', '1']:
    os.environ['SRNN_L1_LDS'] = mode
    out = torch.empty(B * Tl, D, device=DEV, dtype=torch.bfloat16)
    H.lib().call('srnn_mlp_l1', H.BF16, H.ptr(tab), H.ptr(x), x.shape[1], 0, B, Tl, H.BF16,
                 H.ptr(up), D, H.ptr(out), D, D, FS0, Q, H.stream())
    idx = torch.stack([x[:, k:k + Tl] for k in range(FS0)], -1).reshape(B * Tl, FS0)
    pre = up.float().clone()
    for k in range(FS0):
        pre += tab[k].float()[idx[:, k]]
    ref = pre.clamp_min(0)
    err = (out.float() - ref).abs()
    print('mode', mode, 'max err', err.max().item())
    bad = (err > 0.05).nonzero()
    print('bad count', bad.shape[0], 'first', bad[:5].tolist())
    if bad.shape[0]:
        r, c = bad[0].tolist()
        print('out', out[r, c].item(), 'ref', ref[r, c].item(), 'pre', pre[r, c].item(),
              'up', up[r, c].item())
        rows = bad[:, 0].unique()
        cols = bad[:, 1].unique()
        print('bad rows', rows[:20].tolist(), 'n', rows.numel(), 'bad cols', cols[:40].tolist(), cols.numel())
