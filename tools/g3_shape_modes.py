"""Times the TBPTT step's largest GEMMs (layouts, epilogues and dtypes as in model.py) under
the gemm3 variant SRNN_G3MODE selects (read once per process):
  for m in 2 0 1 3 4; do SRNN_G3MODE=$m python tools/g3_shape_modes.py; done"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
import samplernn_hip as H  # noqa: E402

DEV = 'cuda'
bf = torch.bfloat16
g = torch.Generator(device=DEV).manual_seed(0)


def r(*s, dt=bf):
    return (torch.randn(*s, device=DEV, generator=g) * 0.05).to(dt)


M, D, Q = 131072, 1024, 256
a1, a2, da2, W = r(M, D), r(M, D), r(M, D), r(D, D)
mask = torch.relu(r(M, D))
Mb, k = 8192, 16
outsT, dYT, Wup = r(Mb, D), r(Mb, k * D), r(k * D, D)
bias = torch.zeros(D, device=DEV)
cases = {
    'hid_fwd NT 131072x1024x1024 bias+relu bf16': lambda: H.linear(a1, W, bias=bias, relu=True,
                                                                  out_dtype=bf),
    'da1 NN 131072x1024x1024 mask bf16': lambda: H.gemm(da2, W, mask=mask, out_dtype=bf),
    'dW_hid TN 1024x1024x131072 fp32': lambda: H.gemm(da2, a1, transA=True),
    'dWupT TN 1024x16384x8192 fp32': lambda: H.gemm(outsT, dYT, transA=True),
    'dX NN 8192x1024x16384 fp32': lambda: H.gemm(dYT, Wup),
    'up_fwd NT 8192x16384x1024 bf16': lambda: H.linear(outsT, Wup, out_dtype=bf),
}
if os.environ.get('SPLITK_NN') == '1':
    dGI, Wih = r(8192, 3 * D), r(3 * D, D)
    dYt, Wt = r(2048, 4 * D), r(4 * D, D)
    dGIt = r(2048, 3 * D)
    cases = {
        'dX NN 8192x1024x16384 fp32': lambda: H.gemm(dYT, Wup),
        'gru dX NN 8192x1024x3072 fp32': lambda: H.gemm(dGI, Wih),
        'top dX NN 2048x1024x4096 fp32': lambda: H.gemm(dYt, Wt),
        'top gru dX NN 2048x1024x3072 fp32': lambda: H.gemm(dGIt, Wih),
    }
mode = os.environ.get('SRNN_G3MODE', '2')
for name, fn in cases.items():
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / 10 * 1e3)
    print('mode %s  %-46s %8.1f us' % (mode, name, best), flush=True)
