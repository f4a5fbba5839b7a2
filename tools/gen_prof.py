"""One configs[2] generation run (128 utterances x 750 cond rows, dim 1024) in the given dtype,
for rocprofv3 kernel traces: python tools/gen_prof.py fp32|bf16 [n_cond]."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
import torch  # noqa: E402
import bench  # noqa: E402

dt = torch.float32 if sys.argv[1] == 'fp32' else torch.bfloat16
n_cond = int(sys.argv[2]) if len(sys.argv) > 2 else 750
t, _ = bench.run_gen(torch.device('cuda', 0), 128, n_cond, dt)
print('gen %s: %.3f s for %d samples/row' % (sys.argv[1], t, n_cond * 64))
