"""Does replaying the SAME HIP graph back to back expose a host gap per replay?  A graph of
NK small kernels (plus a 4-B pre-copy outside the graph, as Trainer._graph_step does) is
replayed R times: one graph exec vs two identical execs alternated.  Reports wall time per
replay, host time inside replay(), and the GPU's own time per replay (events)."""
import time

import torch

NK, R = 150, 40
dev = 'cuda'
x = torch.zeros(1 << 16, device=dev)
src = torch.ones(1, device=dev)
dst = torch.zeros(1, device=dev)


def body():
    for _ in range(NK):
        x.add_(1.0)


def capture():
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            body()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    return g


gs = [capture(), capture()]
for mode in ('one', 'two', 'one', 'two'):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t_in = 0.0
    t0 = time.perf_counter()
    e0.record()
    for r in range(R):
        dst.copy_(src)
        g = gs[0] if mode == 'one' else gs[r % 2]
        t1 = time.perf_counter()
        g.replay()
        t_in += time.perf_counter() - t1
    e1.record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / R * 1e6
    print('%-4s graphs: wall %.1f us/replay, host in replay() %.1f us, GPU %.1f us/replay'
          % (mode, wall, t_in / R * 1e6, e0.elapsed_time(e1) / R * 1e3), flush=True)
# the GPU time of the body alone (kernels back to back, eager)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for r in range(R):
    body()
e1.record()
torch.cuda.synchronize()
print('eager body: GPU %.1f us per %d kernels' % (e0.elapsed_time(e1) / R * 1e3, NK))
