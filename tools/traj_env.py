"""Chaos check of the 50-chunk bf16 TBPTT trajectory (tests/test_gpu_parity_big.py::
test_bf16_loss_trajectory_50_chunks): the fp32 trajectory, the bf16 one with and without the
log-softmax epilogue (SRNN_LSM_EPI), and bf16 runs from weights perturbed by one ulp (random
signs, two seeds) -- the trajectory's own sensitivity to a rounding-level change.
Prints per run: max / mean relative loss difference vs fp32 (and the chunk of the max), final
loss; and the max distance between bf16 runs."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))
import bench  # noqa: E402
import nn as snn  # noqa: E402
import optim  # noqa: E402

DEV = 'cuda'
B, T, L, N = 128, 1024, 64, 50
batches = bench.gpu_batches(bench.synth_batches(B, T, L, N, 0), DEV)


def traj(dtype, lsm=True, ulp_seed=None):
    os.environ['SRNN_LSM_EPI'] = '1' if lsm else '0'
    _, pred = bench.make_model(dtype)
    if ulp_seed is not None:
        g = torch.Generator().manual_seed(ulp_seed)
        with torch.no_grad():
            for p in pred.parameters():
                s = torch.randint(0, 2, p.shape, generator=g) * 2 - 1
                p.copy_(torch.nextafter(p, p + s.to(p.dtype) * float('inf')))
    pred = pred.to(DEV)
    opt = optim.gradient_clipping(torch.optim.Adam(pred.parameters(), lr=1e-3))
    out = []
    for inp, reset, tgt, cnd, spk in batches:
        opt.zero_grad()

        def closure():
            loss = snn.sequence_nll_loss_bits(pred(inp, reset, cnd, spk), tgt)
            loss.backward()
            return loss
        out.append(opt.step(closure).detach())
    return torch.stack(out).double().cpu().numpy()


b = traj(torch.float32)
runs = {'bf16 lsm': traj(torch.bfloat16, True), 'bf16 no-lsm': traj(torch.bfloat16, False),
        'bf16 lsm ulp1': traj(torch.bfloat16, True, 1), 'bf16 lsm ulp2': traj(torch.bfloat16, True, 2)}
print('fp32: %.4f -> %.4f' % (b[0], b[-1]))
for k, a in runs.items():
    rel = np.abs(a - b) / np.abs(b)
    print('%-14s vs fp32: max rel %.3g (chunk %d), mean rel %.3g, final %.4f'
          % (k, rel.max(), int(rel.argmax()), rel.mean(), a[-1]))
ks = list(runs)
for i in range(len(ks)):
    for j in range(i + 1, len(ks)):
        d = np.abs(runs[ks[i]] - runs[ks[j]]) / np.abs(b)
        print('%-14s vs %-14s: max %.3g (chunk %d)' % (ks[i], ks[j], d.max(), int(d.argmax())))
