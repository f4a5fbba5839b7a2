"""Generation throughput (configs[2]: 3-tier dim 1024 FS=[16,4], B utterances x n_cond rows)
for both sample-loop paths and dtypes.  python tools/gen_bench.py [B] [n_cond]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    n_cond = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    import model as M
    import samplernn_hip as H
    for dt in (torch.bfloat16, torch.float32):
        m, _ = bench.make_model(dt, seed=4242)
        m = m.to(dev)
        cond = torch.rand(B, n_cond, 43, generator=torch.Generator().manual_seed(1))
        spk = np.arange(B) % 6
        for persistent in (True, False):
            gen = M.Generator(m, True)
            gen(B, 0, cond[:, :4], spk, sampler='philox', seed=5, persistent=persistent)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            gen(B, 0, cond, spk, sampler='philox', seed=5, persistent=persistent)
            torch.cuda.synchronize()
            t = time.perf_counter() - t0
            steps = n_cond * 64
            print('%s persistent=%d (rows/group %d): %.1f us/step, %.0f samples/s = %.1fx '
                  'real time' % (dt, persistent, H.gen_persistent_rows(dt, B, 1024, 16),
                                 t / steps * 1e6, B * steps / t, B * steps / t / 16000),
                  flush=True)


if __name__ == '__main__':
    main()
