"""Short bf16 generation run for rocprofv3 kernel traces (configs[2] shapes, B=128)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    n_cond = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    persistent = (sys.argv[3] != '0') if len(sys.argv) > 3 else True
    dt = torch.bfloat16 if (len(sys.argv) <= 4 or sys.argv[4] == 'bf16') else torch.float32
    torch.cuda.set_device(0)
    import model as M
    m, _ = bench.make_model(dt, seed=4242)
    m = m.to('cuda')
    cond = torch.rand(B, n_cond, 43, generator=torch.Generator().manual_seed(1))
    gen = M.Generator(m, True)
    gen(B, 0, cond, np.arange(B) % 6, sampler='philox', seed=5, persistent=persistent)
    torch.cuda.synchronize()
    if os.environ.get('SRNN_GEN_DIAG'):
        import samplernn_hip as H
        H.lib().dll.srnn_gen_diag_dump()


if __name__ == '__main__':
    main()
