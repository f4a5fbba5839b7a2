"""Host-side cost of the eager TBPTT step (the path data-parallel training runs, graph mode
being off under DP): cProfile over eager Trainer.train chunks at ROWS rows.

  SRNN_GRAPH=0 python tools/host_prof.py [rows] [steps]  > gpurun_out/host_prof.txt

SRNN_DP_FORCE=1 adds the data-parallel gradient hook over a one-rank RCCL group (as
bench.py does); SRNN_GRAPH=1 profiles the graph replays instead of eager steps.
"""
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault('SRNN_GRAPH', '0')

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    import nn as snn
    import optim
    from trainer import Trainer
    dev = torch.device('cuda', 0)
    m, pred = bench.make_model(torch.bfloat16)
    pred = pred.to(dev)
    sync = None
    if os.environ.get('SRNN_DP_FORCE', '0') == '1':
        import distributed as D
        D.init()
        sync = D.GradAllReduce(overlap_groups=D.readiness_groups(pred))
    opt = optim.gradient_clipping(torch.optim.Adam(pred.parameters(), lr=1e-3), grad_sync=sync)
    batches = bench.gpu_batches(bench.synth_batches(rows, bench.T_SEQ, 64, 3 + steps, 0), dev)
    tr = Trainer(pred, snn.sequence_nll_loss_bits, opt, batches[:3], True, None)
    tr.train()
    torch.cuda.synchronize()
    tr.dataset = batches[3:]
    tr.enqueue_s = 0.0
    t0 = time.perf_counter()
    tr.train()
    torch.cuda.synchronize()
    print('rows %d, no profiler: %.3f ms/step wall, host enqueue %.3f ms/step'
          % (rows, (time.perf_counter() - t0) / steps * 1e3, tr.enqueue_s / steps * 1e3))
    tr.enqueue_s = 0.0
    # the backward's Python functions run on the calling thread (visible to cProfile)
    torch.autograd.set_multithreading_enabled(False)
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    tr.train()
    pr.disable()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print('rows %d: %.3f ms/step wall, host enqueue %.3f ms/step (graph steps %d)'
          % (rows, dt / steps * 1e3, tr.enqueue_s / steps * 1e3, tr.graph_steps))
    for key in ('tottime', 'cumulative'):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(70)
        print(s.getvalue())


if __name__ == '__main__':
    main()
