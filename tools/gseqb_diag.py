"""Diagnose persistent GRU backward vs per-step vs torch at the last step."""
import torch, sys
sys.path.insert(0, '.')
import importlib
H = importlib.import_module('jalil-saboorizadeh-multi-speaker-neural-vocoder_amd.samplernn_hip')
DEV = 'cuda'
B, D, Fr = 128, 1024, 4
T = torch.bfloat16
g = torch.Generator().manual_seed(3)
whh = (torch.randn(3 * D, D, generator=g) * 0.03).to(DEV, T)
whhT = whh.t().contiguous()
gt = torch.rand(B, Fr, 4 * D, generator=g).to(DEV)
out = torch.randn(B, Fr, D, generator=g).to(DEV)
h0 = torch.randn(B, D, generator=g).to(DEV)
dy = (torch.randn(B, Fr, D, generator=g) * 0.1).to(DEV)
res = {}
for mode in ('seq', 'steps'):
    dgh = torch.zeros((B, Fr, 3 * D), device=DEV)
    dghT = torch.zeros((B, Fr, 3 * D), device=DEV, dtype=T)
    dgi = torch.zeros((B, Fr, 3 * D), device=DEV)
    ddir = [torch.zeros(B, D, device=DEV) for _ in range(2)]
    if mode == 'seq':
        nw = 64 * ((B + 31) // 32) + 1
        work = torch.zeros((nw,), device=DEV, dtype=torch.int32)
        H.lib().call('srnn_gru_seq_bwd', H.BF16, B, D, Fr, H.ptr(dy), Fr * D, D,
                     H.ptr(gt), Fr * 4 * D, 4 * D, H.ptr(out), Fr * D, D, H.ptr(h0),
                     H.ptr(whhT), H.ptr(dgh), H.ptr(dghT), H.ptr(dgi), Fr * 3 * D,
                     3 * D, H.ptr(ddir[0]), H.ptr(work), nw * 4, H.stream())
    else:
        for t in reversed(range(Fr)):
            nxt = t + 1 < Fr
            hp, ldhp = (out[:, t - 1], Fr * D) if t > 0 else (h0, D)
            H.lib().call('srnn_gru_cell_bwd', H.BF16, B, D, H.ptr(dy[:, t]), Fr * D,
                         H.ptr(dghT[:, t + 1]) if nxt else None, Fr * 3 * D,
                         H.ptr(ddir[(t + 1) % 2]) if nxt else None, H.ptr(whh),
                         H.ptr(whhT), H.ptr(gt[:, t]), Fr * 4 * D, H.ptr(hp), ldhp,
                         H.ptr(dgh[:, t]), Fr * 3 * D, H.ptr(dghT[:, t]), Fr * 3 * D,
                         H.ptr(dgi[:, t]), Fr * 3 * D, H.ptr(ddir[t % 2]), H.stream())
    torch.cuda.synchronize()
    res[mode] = dgh
t = Fr - 1
r, z, n, ghn = gt[:, t].split(D, 1)
dh = dy[:, t]
hp = out[:, t - 1]
dn = dh * (1 - z); dz = dh * (hp - n); dan = dn * (1 - n * n)
dar = dan * ghn * r * (1 - r); daz = dz * z * (1 - z); dghn = dan * r
ref = torch.cat([dar, daz, dghn], 1)
for m in res:
    d = (res[m][:, t] - ref).abs()
    print(m, [float(x.max()) for x in d.split(D, 1)])
d = (res['seq'] - res['steps']).abs()
for t in range(Fr):
    print('t', t, [float(x.max()) for x in d[:, t].split(D, 1)], int((d[:, t] != 0).sum()))
