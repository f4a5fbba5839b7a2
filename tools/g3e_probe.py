"""gemm3e (8-phase ping-pong NT kernel, SRNN_G3E=1) against the pair-mode gemm3p
(SRNN_G3E=0) and hipBLASLt (the default routing) on the TBPTT step's NT GEMMs at B = 512 with
their epilogues, interleaved in one process (uniform random bf16 operands, min / median of
rounds x reps, HIP events).  gemm3e must equal gemm3p bit for bit (same k order)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..',
                                'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
import samplernn_hip as H  # noqa: E402

ROUNDS = int(os.environ.get('ROUNDS', '4'))
REPS = int(os.environ.get('REPS', '5'))


def bench(fn, reps=REPS):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def variant(v):
    os.environ['SRNN_BLASLT'] = '1' if v == 'blaslt' else '0'
    os.environ['SRNN_G3E'] = '1' if v == 'g3e' else '0'


M = int(os.environ.get('ROWS', '512')) * 1024
bf = torch.bfloat16
# name, M, N, K, out dtype, bias, relu, bits_out
shapes = [('hid_fwd', M, 1024, 1024, bf, True, True, True),
          ('up_fwd', M // 16, 16384, 1024, bf, True, False, False),
          ('out_fwd', M, 256, 1024, torch.float32, True, False, False),
          ('gi_fwd', M // 16, 3072, 1024, torch.float32, True, False, False),
          ('plain_bf16', M // 4, 1024, 1024, bf, False, False, False),
          # the da2 GEMM's shape (K = Q = 256: 4 k-tiles per output tile, epilogue-heavy)
          ('k256_bf16', M, 1024, 256, bf, False, False, False),
          ('k256_bits', M, 1024, 256, bf, True, True, True)]
ONLY = [x for x in os.environ.get('ONLY', '').split(',') if x]
if ONLY:
    shapes = [sh for sh in shapes if sh[0] in ONLY]
g = torch.Generator(device='cuda').manual_seed(5)
res = {}
for name, m, n, k, od, hb, relu, bo in shapes:
    a = (torch.rand(m, k, device='cuda', generator=g) * 2 - 1).to(bf)
    w = (torch.rand(n, k, device='cuda', generator=g) * 2 - 1).to(bf)
    bias = (torch.rand(n, device='cuda', generator=g) - 0.5) if hb else None
    outs = {}
    for v in ('g3p', 'g3e', 'blaslt'):
        variant(v)
        bits = H.relu_bits(m, n, 'cuda') if bo and v != 'blaslt' else None
        o = H.gemm(a, w, transB=True, out_dtype=od, bias=bias, relu=relu, bits_out=bits)
        torch.cuda.synchronize()
        outs[v] = (o, bits)
    same = torch.equal(outs['g3p'][0], outs['g3e'][0])
    bsame = (outs['g3p'][1] is None) or torch.equal(outs['g3p'][1], outs['g3e'][1])
    ref = outs['blaslt'][0].float()
    err = (outs['g3e'][0].float() - ref).abs().max().item()
    print('%-10s %7dx%5dx%5d  g3e==g3p %s bits %s  max|g3e-blaslt| %.3g' % (
        name, m, n, k, same, bsame, err), flush=True)
    res[name] = {v: [] for v in ('g3p', 'g3e', 'blaslt')}
    for r in range(ROUNDS):
        for v in ('g3p', 'g3e', 'blaslt'):
            variant(v)
            bits = outs[v][1]
            out = outs[v][0]
            res[name][v].append(bench(lambda: H.gemm(a, w, transB=True, out=out, out_dtype=od,
                                                      bias=bias, relu=relu, bits_out=bits)))
    line = '%-10s %7dx%5dx%5d' % (name, m, n, k)
    for v in ('g3p', 'g3e', 'blaslt'):
        ts = sorted(res[name][v])
        tf = 2.0 * m * n * k / (ts[0] * 1e-6) / 1e12
        line += '  %s %8.1f us (med %8.1f, %5.0f TF/s)' % (v, ts[0], ts[len(ts) // 2], tf)
    print(line, flush=True)
    del a, w, outs
variant('blaslt')
