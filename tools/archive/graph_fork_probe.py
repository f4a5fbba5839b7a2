"""Do the parallel branches of a captured HIP graph run concurrently?  Main stream and a
forked side stream each run a spin kernel (torch.cuda._sleep) and, in the second case, a
64-row persistent GRU sweep on main beside a bf16 GEMM pair on the side:  replay times of
the forked graph vs the same work serial.   python tools/graph_fork_probe.py"""
import os
import sys
import time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..',
                                'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
import torch  # noqa: E402
import samplernn_hip as H  # noqa: E402

dev = torch.device('cuda', 0)


def replay_ms(g, n=20):
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def capture(fn):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        fn()
    torch.cuda.synchronize()
    return g


side = torch.cuda.Stream()


def forked(a, b):
    def f():
        main = torch.cuda.current_stream()
        side.wait_stream(main)
        with torch.cuda.stream(side):
            b()
        a()
        main.wait_stream(side)
    return f


CYC = 2000000
sl = lambda: torch.cuda._sleep(CYC)   # noqa: E731
print('sleep serial   %.3f ms' % replay_ms(capture(lambda: (sl(), sl()))))
print('sleep forked   %.3f ms' % replay_ms(capture(forked(sl, sl))))

# a 64-row bf16 XCD sweep (half the chip) beside two bf16 GEMMs
B, D, Fr = 64, 1024, 64
T = torch.bfloat16
g0 = torch.Generator().manual_seed(1)
whh = (torch.randn(3 * D, D, generator=g0) * 0.03).to(dev, T)
bhh = (torch.randn(3 * D, generator=g0) * 0.1).to(dev)
gi = (torch.randn(B, Fr, 3 * D, generator=g0) * 0.5).to(dev)
h0 = (torch.randn(B, D, generator=g0) * 0.5).to(dev)
nf = H.gru_xcd_work_bytes(T, B, D)
wf = torch.empty(nf, device=dev, dtype=torch.uint8)
out = torch.empty((B, Fr, D), device=dev)
outT = torch.empty((B, Fr, D), device=dev, dtype=T)
gt = torch.empty((B, Fr, 4 * D), device=dev)
hp = torch.empty((B, Fr, D), device=dev, dtype=T)
x = torch.randn(4096, 4096, device=dev).to(T)
y = torch.randn(4096, 4096, device=dev).to(T)
z = torch.empty(4096, 4096, device=dev, dtype=T)


def sweep():
    H.lib().call('srnn_gru_xcd_fwd2', H.BF16, B, D, Fr, H.ptr(gi), Fr * 3 * D, 3 * D,
                 H.ptr(h0), H.ptr(whh), H.ptr(bhh), H.ptr(out), H.ptr(outT), Fr * D, D,
                 H.ptr(gt), Fr * 4 * D, 4 * D, H.ptr(hp), H.ptr(wf), nf, H.stream())


def gemms():
    for _ in range(3):
        torch.mm(x, y, out=z)


print('sweep alone    %.3f ms' % replay_ms(capture(sweep)))
print('gemms alone    %.3f ms' % replay_ms(capture(gemms)))
print('serial         %.3f ms' % replay_ms(capture(lambda: (sweep(), gemms()))))
print('forked         %.3f ms' % replay_ms(capture(forked(sweep, gemms))))
ref = out.clone()
torch.cuda.synchronize()
assert H.lib().dll.srnn_gru_xcd_error(H.ptr(wf)) == 0
H.check_persistent_errors()
print('sweep error flag clear')
