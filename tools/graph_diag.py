"""Run-to-run spread of the TBPTT step (eager x3, then graph mode): which runs agree bit for
bit (graph-mode test tolerance)."""
import sys
import os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'tests'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
import conftest  # noqa: F401  (sys.path for the package)
import torch
import bench
import test_gpu_graph as TG

dt = torch.float32 if sys.argv[1:] == ['fp32'] else torch.bfloat16
raw = bench.synth_batches(64, 1024, 64, 8, 0)
raw = [(a, n % 4 == 0, t, c, s) for n, (a, _, t, c, s) in enumerate(raw)]
batches = bench.gpu_batches(raw, 'cuda')
names = ('eager1', 'eager2', 'eager3', 'graph')
runs = [TG._train(dt, batches, g)[:2] for g in (False, False, False, True)]
for i in range(4):
    for j in range(i + 1, 4):
        li, pi = runs[i]
        lj, pj = runs[j]
        worst = max(((pi[k] - pj[k]).abs().max().item(), k) for k in pi)
        print(names[i], names[j], 'loss diff', max(abs(a - b) for a, b in zip(li, lj)),
              'worst param', worst)
