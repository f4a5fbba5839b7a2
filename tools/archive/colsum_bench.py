"""Time srnn_colsum (samplernn_hip.colsum) on the TBPTT step's two bf16 column sums at B = 512:
db_hid = colsum(da2) over (524288, 1024) and db_out = colsum(dz) over (524288, 256); HIP
events around 10 back-to-back calls after 3 warm-ups; bytes read / time."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..',
                                'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
import samplernn_hip as H  # noqa: E402

for rows, cols in ((524288, 1024), (524288, 256), (131072, 1024)):
    x = torch.randn(rows, cols, device='cuda').bfloat16()
    out = torch.empty(cols, device='cuda')
    for _ in range(3):
        H.colsum(x, rows, cols, out=out)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        H.colsum(x, rows, cols, out=out)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / 10
    ref = x.float().sum(0)
    err = ((out - ref).abs().max() / ref.abs().max()).item()
    print('colsum %d x %d bf16: %.1f us, %.2f TB/s, max rel err %.2e'
          % (rows, cols, ms * 1e3, rows * cols * 2 / ms / 1e9, err), flush=True)
