"""Microbenchmark of libsamplernn_hip GEMM shapes used by the TBPTT step (HIP events)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
import samplernn_hip as H  # noqa: E402

DEV = 'cuda'


def timeit(fn, reps=30):
    for _ in range(10):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def run(M, N, K, tA, tB, dtype, out_dtype, tile, tag):
    A = torch.randn(K, M, device=DEV).to(dtype) if tA else torch.randn(M, K, device=DEV).to(dtype)
    B = torch.randn(N, K, device=DEV).to(dtype) if tB else torch.randn(K, N, device=DEV).to(dtype)
    out = torch.empty(M, N, device=DEV, dtype=out_dtype)
    kw = {}
    if '+mask' in tag:
        kw['mask'] = torch.randn(M, N, device=DEV).to(dtype)
    if '+bias' in tag:
        kw['bias'] = torch.randn(N, device=DEV)
        kw['relu'] = True
    ms = timeit(lambda: H.gemm(A, B, transA=tA, transB=tB, out=out, tile=tile, **kw))
    tf = 2.0 * M * N * K / ms / 1e9
    print('%-34s tile=%2d %7.3f ms %8.1f TFLOP/s' % (tag, tile, ms, tf), flush=True)


def run_torch(M, N, K, tA, tB, dtype, tag):
    """the vendor library (hipBLASLt / rocBLAS through torch.mm) on the same shape, for scale"""
    A = torch.randn(K, M, device=DEV).to(dtype) if tA else torch.randn(M, K, device=DEV).to(dtype)
    B = torch.randn(N, K, device=DEV).to(dtype) if tB else torch.randn(K, N, device=DEV).to(dtype)
    a = A.t() if tA else A
    b = B.t() if tB else B
    out = torch.empty(M, N, device=DEV, dtype=dtype)
    ms = timeit(lambda: torch.mm(a, b, out=out))
    print('%-34s torch   %7.3f ms %8.1f TFLOP/s' % (tag, ms, 2.0 * M * N * K / ms / 1e9), flush=True)


if __name__ == '__main__':
    bf, f32 = torch.bfloat16, torch.float32
    shapes = [
        (131072, 1024, 1024, False, True, bf, bf, 'mlp hidden fwd NT'),
        (131072, 256, 1024, False, True, bf, f32, 'mlp out fwd NT'),
        (131072, 1024, 1024, False, False, bf, f32, 'mlp dgrad NN'),
        (1024, 1024, 131072, True, False, bf, f32, 'mlp wgrad TN'),
        (8192, 16384, 1024, False, True, bf, f32, 'upsample fwd NT'),
        (8192, 1024, 16384, False, False, bf, f32, 'upsample dgrad NN'),
        (16384, 1024, 8192, True, False, bf, f32, 'upsample wgrad TN'),
        (8192, 3072, 1024, False, True, bf, f32, 'gru gi fwd NT'),
        (3072, 1024, 8192, True, False, bf, f32, 'gru wgrad TN'),
        (131072, 1024, 256, False, False, bf, bf, 'mlp dgrad out NN K256'),
        (131072, 1024, 1024, False, True, bf, f32, 'mlp hidden fwd NT f32out'),
        (131072, 1024, 1024, False, True, bf, bf, 'mlp hidden fwd NT +bias'),
        (131072, 1024, 1024, False, False, bf, f32, 'mlp dgrad NN +mask'),
        (131072, 1024, 256, False, False, bf, bf, 'mlp dgrad out NN K256 +mask'),
        (16384, 1024, 8192, False, True, bf, f32, 'mlp hidden NT K8192'),
        (131072, 1024, 1024, True, False, bf, bf, 'mlp hidden TN bf16out'),
        (256, 1024, 131072, True, False, bf, f32, 'mlp out wgrad TN'),
        (2048, 3072, 1024, False, True, bf, f32, 'top gi fwd NT'),
        (2048, 4096, 1024, False, True, bf, f32, 'top upsample fwd NT'),
        (2048, 1024, 4096, False, False, bf, f32, 'top upsample dgrad NN'),
        (4096, 1024, 2048, True, False, bf, f32, 'top upsample wgrad TN'),
        (3072, 1024, 2048, True, False, bf, f32, 'top gru wgrad TN'),
        (8192, 1024, 3072, False, False, bf, f32, 'gru dgrad NN'),
    ]
    tiles = [int(t) for t in os.environ.get('TILES', '5,3').split(',')]
    only = os.environ.get('ONLY')
    for (M, N, K, tA, tB, dt, odt, tag) in shapes:
        if only and only not in tag:
            continue
        for tile in tiles:
            run(M, N, K, tA, tB, dt, odt, tile, tag)
        if os.environ.get('TORCHREF') == '1':
            run_torch(M, N, K, tA, tB, dt, tag)
