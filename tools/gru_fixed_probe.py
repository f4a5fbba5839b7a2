"""Fixed vs per-step cost of the persistent GRU sweeps (gru_xcd.hip): each sweep alone at B
rows and Fr = 16 / 64 / 128 frames (bench.gru_sweep_roofline, HIP events), so the per-launch
intercept (prologue: W_hh fragment loads, arrival gate; epilogue) separates from the per-step
hand-off cost.  python3 tools/gru_fixed_probe.py"""
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, '..'))
sys.path.insert(0, os.path.join(HERE, '..', 'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
import bench  # noqa: E402

dev = torch.device('cuda', 0)
print('SRNN_GX_EXP=%s' % os.environ.get('SRNN_GX_EXP', '0'), flush=True)
for B in (64, 512):
    pts = {}
    for Fr in (16, 64, 128):
        r = bench.gru_sweep_roofline(dev, B=B, Fr=Fr, reps=10)
        pts[Fr] = {k: r[k]['us_per_step'] * Fr for k in ('fwd', 'bwd')}
        print('B %d Fr %3d: fwd %.1f us, bwd %.1f us per sweep' % (B, Fr, pts[Fr]['fwd'],
                                                                   pts[Fr]['bwd']), flush=True)
    for k in ('fwd', 'bwd'):
        slope = (pts[128][k] - pts[16][k]) / 112.0
        print('B %d %s: %.2f us per step, intercept %.1f us' % (B, k, slope, pts[16][k] - 16 * slope),
              flush=True)
