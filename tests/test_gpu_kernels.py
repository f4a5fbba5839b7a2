"""Op-level parity of the HIP kernels (through the C ABI) on an MI355X.

Floating-point kernels are checked against a plain PyTorch fp32 reference of the same op;
the mu-law quantiser is checked bit-exactly against the reference-derived staircase.
"""
import ctypes

import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu

DEV = 'cuda'


def _rand(*shape, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(*shape, generator=g) * 2 - 1) * scale


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('transA,transB', [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize('tile', [0, 1, 2])
@pytest.mark.parametrize('M,N,K', [(37, 53, 29), (130, 260, 70), (256, 128, 1024)])
def test_gemm_layouts(hip, dtype, transA, transB, tile, M, N, K):
    A = _rand(K, M, seed=1) if transA else _rand(M, K, seed=1)
    B = _rand(N, K, seed=2) if transB else _rand(K, N, seed=2)
    bias = _rand(N, seed=3)
    cin = _rand(M, N, seed=4)
    Ad, Bd = A.to(DEV, dtype), B.to(DEV, dtype)
    out = hip.gemm(Ad, Bd, transA=bool(transA), transB=bool(transB), bias=bias.to(DEV),
                   cin=cin.to(DEV), beta=0.5, alpha=1.5, relu=True, tile=tile)
    Af, Bf = Ad.float().cpu(), Bd.float().cpu()
    ref = 1.5 * ((Af.t() if transA else Af) @ (Bf.t() if transB else Bf)) + 0.5 * cin + bias
    ref = ref.clamp_min(0)
    tol = 1e-4 * np.sqrt(K) if dtype == torch.float32 else 2e-3 * np.sqrt(K)
    torch.testing.assert_close(out.cpu(), ref, atol=tol, rtol=1e-4)


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('transA,transB', [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize('M,N,K,epi', [(256, 384, 512, True), (384, 128, 256, True),
                                       (128, 256, 8192, False)])
def test_gemm2_ring_kernel(hip, dtype, transA, transB, M, N, K, epi):
    """The glds-ring kernel (tile 3 forces it): all layouts, epilogue and split-K paths."""
    A = _rand(K, M, seed=1) if transA else _rand(M, K, seed=1)
    B = _rand(N, K, seed=2) if transB else _rand(K, N, seed=2)
    Ad, Bd = A.to(DEV, dtype), B.to(DEV, dtype)
    Af, Bf = Ad.float().cpu(), Bd.float().cpu()
    ref = (Af.t() if transA else Af) @ (Bf.t() if transB else Bf)
    if epi:
        bias = _rand(N, seed=3)
        cin = _rand(M, N, seed=4)
        out = hip.gemm(Ad, Bd, transA=bool(transA), transB=bool(transB), bias=bias.to(DEV),
                       cin=cin.to(DEV), beta=0.5, relu=True, tile=3)
        ref = (ref + 0.5 * cin + bias).clamp_min(0)
    else:   # plain fp32 output with few tiles -> split-K with atomics
        out = hip.gemm(Ad, Bd, transA=bool(transA), transB=bool(transB), tile=3)
    tol = 1e-4 * np.sqrt(K) if dtype == torch.float32 else 2e-3 * np.sqrt(K)
    torch.testing.assert_close(out.cpu(), ref, atol=tol, rtol=1e-4)


@pytest.mark.parametrize('out_dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('transA,transB', [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize('M,N,K,epi', [(512, 768, 320, 'full'), (256, 512, 96, 'rowbias'),
                                       (256, 256, 8192, 'plain'), (768, 256, 1024, 'plain')])
def test_gemm3_256_kernel(hip, out_dtype, transA, transB, M, N, K, epi):
    """The 256x256 8-wave bf16 kernel (tile 5 forces it): all layouts, vectorised epilogue
    (Cin, column/row bias, ReLU, mask) and the split-K atomic path."""
    dtype = torch.bfloat16
    A = _rand(K, M, seed=1) if transA else _rand(M, K, seed=1)
    B = _rand(N, K, seed=2) if transB else _rand(K, N, seed=2)
    Ad, Bd = A.to(DEV, dtype), B.to(DEV, dtype)
    Af, Bf = Ad.float().cpu(), Bd.float().cpu()
    ref = (Af.t() if transA else Af) @ (Bf.t() if transB else Bf)
    kw = dict(transA=bool(transA), transB=bool(transB), tile=5, out_dtype=out_dtype)
    if epi == 'full':
        bias, cin, mask = _rand(N, seed=3), _rand(M, N, seed=4), _rand(M, N, seed=5)
        out = hip.gemm(Ad, Bd, bias=bias.to(DEV), cin=cin.to(DEV), beta=0.5, relu=True,
                       mask=mask.to(DEV, dtype), alpha=1.5, **kw)
        ref = (1.5 * ref + 0.5 * cin + bias).clamp_min(0) * (mask.to(dtype).float() > 0)
    elif epi == 'rowbias':
        bias = _rand(M, seed=3)
        out = hip.gemm(Ad, Bd, bias=bias.to(DEV), bias_mode=2, **kw)
        ref = ref + bias[:, None]
    else:
        out = hip.gemm(Ad, Bd, **kw)
    tol = 2e-3 * np.sqrt(K) if out_dtype == torch.float32 else 1e-2 * np.sqrt(K)
    torch.testing.assert_close(out.float().cpu(), ref, atol=tol, rtol=1e-2)


@pytest.mark.parametrize('out_dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('epi', ['plain', 'bias_relu', 'cin'])
def test_gemm3_nn_ring_pingpong(hip, monkeypatch, out_dtype, epi):
    """NN shapes with two rounds of 256x256 tiles take gemm3's ring ping-pong schedule
    (gemm3q_kernel) on the hand-written path: the same MFMA order as the pair schedule
    (SRNN_G3_NNQ=0), so the same bits, and the fp32 product of the bf16 operands."""
    dtype = torch.bfloat16
    M, N, K = 8192, 4096, 512                  # 32 x 16 = 512 tiles, K-contiguous A, N-major B
    A, B = _rand(M, K, seed=1), _rand(K, N, seed=2)
    Ad, Bd = A.to(DEV, dtype), B.to(DEV, dtype)
    ref = Ad.float().cpu() @ Bd.float().cpu()
    kw = dict(tile=5, out_dtype=out_dtype)
    if epi == 'bias_relu':
        bias = _rand(N, seed=3)
        kw.update(bias=bias.to(DEV), relu=True)
        ref = (ref + bias).clamp_min(0)
    elif epi == 'cin':
        cin = _rand(M, N, seed=4)
        kw.update(cin=cin.to(DEV), beta=0.5)
        ref = ref + 0.5 * cin

    def run(q):
        monkeypatch.setenv('SRNN_G3_NNQ', '1' if q else '0')
        out = hip.gemm(Ad, Bd, **kw)
        torch.cuda.synchronize()
        return out.float().cpu()
    q, pair = run(True), run(False)
    assert torch.equal(q, pair)
    tol = 2e-3 * np.sqrt(K) if out_dtype == torch.float32 else 1e-2 * np.sqrt(K)
    torch.testing.assert_close(q, ref, atol=tol, rtol=1e-2)


@pytest.mark.parametrize('out_dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('transA,transB', [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize('M,N,K,epi', [(4096, 2048, 1024, 'bias_relu'), (2048, 4096, 1024, 'bias'),
                                       (4096, 1024, 2048, 'plain')])
def test_gemm_blaslt_plain(hip, monkeypatch, out_dtype, transA, transB, M, N, K, epi):
    """Large plain bf16 GEMMs (alpha, per-column bias, ReLU; beta 0) go to hipBLASLt
    (blaslt.cpp): every layout against the fp32 product of the same bf16 operands, against
    gemm3 (SRNN_BLASLT=0) within bf16 rounding, and bit-identical run to run."""
    dtype = torch.bfloat16
    A = _rand(K, M, seed=1) if transA else _rand(M, K, seed=1)
    B = _rand(N, K, seed=2) if transB else _rand(K, N, seed=2)
    Ad, Bd = A.to(DEV, dtype), B.to(DEV, dtype)
    Af, Bf = Ad.float().cpu(), Bd.float().cpu()
    ref = 1.25 * ((Af.t() if transA else Af) @ (Bf.t() if transB else Bf))
    bias = _rand(N, seed=3)
    kw = dict(transA=bool(transA), transB=bool(transB), out_dtype=out_dtype, alpha=1.25)
    if epi != 'plain':
        kw['bias'] = bias.to(DEV)
        ref = ref + bias
    if epi == 'bias_relu':
        kw['relu'] = True
        ref = ref.clamp_min(0)

    def run(on):
        monkeypatch.setenv('SRNN_BLASLT', '1' if on else '0')
        n0 = hip.lib().dll.srnn_blaslt_calls()
        out = hip.gemm(Ad, Bd, **kw)
        torch.cuda.synchronize()
        assert hip.lib().dll.srnn_blaslt_calls() - n0 == (1 if on else 0)
        return out.float().cpu()
    lt, lt2, g3 = run(True), run(True), run(False)
    assert torch.equal(lt, lt2)
    tol = 2e-3 * np.sqrt(K) if out_dtype == torch.float32 else 1e-2 * np.sqrt(K)
    torch.testing.assert_close(lt, ref, atol=tol, rtol=1e-2)
    torch.testing.assert_close(lt, g3, atol=tol, rtol=1e-2)


@pytest.mark.parametrize('M,N,K,transA,transB,lib', [
    (3072, 1024, 1024, 1, 0, True),      # 64-row step: top-tier W_hh / W_ih gradients
    (1024, 1024, 4096, 0, 0, True),      # top-tier upsampling dX
    (1024, 3072, 1024, 0, 1, True),      # top-tier GRU input projection (with bias below)
    (3072, 1024, 8192, 1, 0, False),     # deep weight gradient: stays on gemm3 split-K
    (256, 1024, 4096, 1, 0, False)])     # under 1 Mi outputs: stays
def test_gemm_route_wide_k(hip, M, N, K, transA, transB, lib):
    """Round-6 routing: plain bf16 products with >= 1 Mi outputs over 256 <= K <= 4096 go to
    hipBLASLt below its old size threshold (blaslt.cpp); deeper or smaller ones stay on the
    hand-written kernels.  Results against the fp32 product of the same operands."""
    A = _rand(K, M, seed=4) if transA else _rand(M, K, seed=4)
    B = _rand(N, K, seed=5) if transB else _rand(K, N, seed=5)
    Ad, Bd = A.to(DEV, torch.bfloat16), B.to(DEV, torch.bfloat16)
    Af, Bf = Ad.float().cpu(), Bd.float().cpu()
    ref = (Af.t() if transA else Af) @ (Bf.t() if transB else Bf)
    kw = dict(transA=bool(transA), transB=bool(transB), out_dtype=torch.float32)
    if transB:
        bias = _rand(N, seed=6)
        kw['bias'] = bias.to(DEV)
        ref = ref + bias
    n0 = hip.lib().dll.srnn_blaslt_calls()
    out = hip.gemm(Ad, Bd, **kw)
    torch.cuda.synchronize()
    assert hip.lib().dll.srnn_blaslt_calls() - n0 == (1 if lib else 0)
    torch.testing.assert_close(out.cpu(), ref, atol=2e-3 * np.sqrt(K), rtol=1e-2)


def test_gemm_route_k64_and_skinny512(hip, monkeypatch):
    """Round-6 routing: the 64-deep input projection over many rows on gemm3 (8192 x 1024 x 64,
    bias, fp32 out) and the 512-row dh_0 product on the skinny kernel (A rows strided, Cin);
    both against the fp32 product of the same operands and against the previous routes."""
    A = _rand(8192, 64, seed=7).to(DEV, torch.bfloat16)
    W = _rand(1024, 64, seed=8).to(DEV, torch.bfloat16)
    b = _rand(1024, seed=9).to(DEV)
    ref = A.float().cpu() @ W.float().cpu().t() + b.cpu()
    out = hip.linear(A, W, bias=b)
    monkeypatch.setenv('SRNN_SMALLK_G3', '0')
    old = hip.gemm(A, W, transB=True, bias=b, tile=6)            # the thin small-K kernel
    monkeypatch.delenv('SRNN_SMALLK_G3')
    torch.cuda.synchronize()
    torch.testing.assert_close(out.cpu(), ref, atol=1e-3, rtol=1e-3)
    torch.testing.assert_close(out.cpu(), old.cpu(), atol=1e-4, rtol=1e-4)
    Fr, D = 4, 1024
    G = _rand(512, Fr, 3 * D, seed=10).to(DEV, torch.bfloat16)
    Wt = _rand(D, 3 * D, seed=11).to(DEV, torch.bfloat16)
    cin = _rand(512, D, seed=12).to(DEV)
    ref = G[:, 0].float().cpu() @ Wt.float().cpu().t() + cin.cpu()
    out = hip.gemm(G[:, 0], Wt, transB=True, M=512, N=D, K=3 * D, lda=Fr * 3 * D, ldb=3 * D,
                   cin=cin, beta=1.0)
    prev = hip.gemm(G[:, 0], Wt, transB=True, M=512, N=D, K=3 * D, lda=Fr * 3 * D, ldb=3 * D,
                    cin=cin, beta=1.0, tile=0)                   # the 128-tile kernel
    torch.cuda.synchronize()
    torch.testing.assert_close(out.cpu(), ref, atol=2e-3 * np.sqrt(3 * D), rtol=1e-2)
    torch.testing.assert_close(out.cpu(), prev.cpu(), atol=2e-3 * np.sqrt(3 * D), rtol=1e-2)


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('transA', [0, 1])
@pytest.mark.parametrize('M,N,K', [(1024, 16, 8192), (1024, 43, 2048), (1000, 6, 128),
                                   (128, 64, 1024), (300, 1, 5000), (1002, 5, 300)])
def test_gemm_thin_small_n(hip, dtype, transA, M, N, K):
    """Thin path (tile 6): N <= 64 weight gradients, split-K (scratch partials or atomics)."""
    A = _rand(K, M, seed=1) if transA else _rand(M, K, seed=1)
    B = _rand(K, N, seed=2)
    Ad, Bd = A.to(DEV, dtype), B.to(DEV, dtype)
    out = hip.gemm(Ad, Bd, transA=bool(transA), tile=6, alpha=0.5)
    Af, Bf = Ad.float().cpu(), Bd.float().cpu()
    ref = 0.5 * ((Af.t() if transA else Af) @ Bf)
    torch.testing.assert_close(out.cpu(), ref, atol=1e-4 * np.sqrt(K), rtol=1e-4)


@pytest.mark.parametrize('dtype,odt', [(torch.float32, torch.float32),
                                       (torch.bfloat16, torch.float32),
                                       (torch.bfloat16, torch.bfloat16)])
@pytest.mark.parametrize('M,N,K', [(8192, 1024, 16), (2048, 1024, 43), (300, 700, 64),
                                   (260, 702, 7)])
def test_gemm_thin_small_k(hip, dtype, odt, M, N, K):
    """Thin path (tile 6): K <= 64 input projections with Cin + bias (+ relu)."""
    A, W = _rand(M, K, seed=1), _rand(N, K, seed=2)
    cin, bias = _rand(M, N, seed=3), _rand(N, seed=4)
    Ad, Wd = A.to(DEV, dtype), W.to(DEV, dtype)
    out = hip.gemm(Ad, Wd, transB=True, cin=cin.to(DEV), beta=1.0, bias=bias.to(DEV), relu=True,
                   out_dtype=odt, tile=6)
    ref = (Ad.float().cpu() @ Wd.float().cpu().t() + cin + bias).clamp_min(0)
    tol = 1e-4 if odt == torch.float32 else 2e-2
    torch.testing.assert_close(out.float().cpu(), ref, atol=tol, rtol=tol)


@pytest.mark.parametrize('B,D,Fr', [(128, 1024, 16), (64, 1024, 5), (100, 256, 9)])
def test_gru_seq_fwd_matches_steps(hip, B, D, Fr):
    """Persistent whole-sequence GRU forward == Fr per-step cell launches, bit for bit."""
    T = torch.bfloat16
    if not hip.gru_seq_supported(T, B, D):
        pytest.skip('persistent GRU not supported on this device')
    g = torch.Generator().manual_seed(B + D)
    whh = (torch.randn(3 * D, D, generator=g) * 0.03).to(DEV, T)
    bhh = (torch.randn(3 * D, generator=g) * 0.1).to(DEV)
    gi = (torch.randn(B * Fr, 3 * D, generator=g) * 0.5).to(DEV)
    h0 = (torch.randn(B, D, generator=g) * 0.5).to(DEV)
    h0T = h0.to(T)
    outs = {}
    for mode in ('seq', 'steps'):
        out = torch.full((B, Fr, D), float('nan'), device=DEV)
        outT = torch.zeros((B, Fr, D), device=DEV, dtype=T)
        gt = torch.full((B, Fr, 4 * D), float('nan'), device=DEV)
        if mode == 'seq':
            nw = 64 * ((B + 31) // 32) + 1
            work = torch.full((nw,), 7, device=DEV, dtype=torch.int32)
            hip.lib().call('srnn_gru_seq_fwd', hip.BF16, B, D, Fr, hip.ptr(gi), Fr * 3 * D, 3 * D,
                           hip.ptr(h0), hip.ptr(h0T), hip.ptr(whh), hip.ptr(bhh), hip.ptr(out),
                           hip.ptr(outT), Fr * D, D, hip.ptr(gt), Fr * 4 * D, 4 * D,
                           hip.ptr(work), work.numel() * 4, hip.stream())
            torch.cuda.synchronize()
            assert int(work[nw - 1]) == 0, 'persistent GRU gave up waiting'
        else:
            for t in range(Fr):
                hp_t, hp_f, ldh = (h0T, h0, D) if t == 0 else (outT[:, t - 1], out[:, t - 1], Fr * D)
                hip.lib().call('srnn_gru_cell', hip.BF16, B, D, D, None, 0, None, None,
                               hip.ptr(gi[t:]), Fr * 3 * D, hip.ptr(hp_t), ldh, hip.ptr(hp_f), ldh,
                               hip.ptr(whh), hip.ptr(bhh), hip.ptr(out[:, t]), Fr * D,
                               hip.ptr(outT[:, t]), Fr * D, hip.ptr(gt[:, t]), Fr * 4 * D,
                               hip.stream())
        outs[mode] = (out.cpu(), outT.float().cpu(), gt.cpu())
    for a, b in zip(outs['seq'], outs['steps']):
        assert torch.equal(a, b)


def _gru_ref(gi, h0, whh, bhh, Fr):
    """torch fp32 GRU recurrence (model.py:148-165, gate order r|z|n) with bf16 W_hh and bf16
    h_{t-1} operands as the MFMA path uses them; fp32 state."""
    B, D = h0.shape
    h = h0.clone()
    out, gates = [], []
    W = whh.float()
    for t in range(Fr):
        gh = h.to(torch.bfloat16).float() @ W.t() + bhh
        g = gi.reshape(B, Fr, 3 * D)[:, t]
        r = torch.sigmoid(gh[:, :D] + g[:, :D])
        z = torch.sigmoid(gh[:, D:2 * D] + g[:, D:2 * D])
        n = torch.tanh(g[:, 2 * D:] + gh[:, 2 * D:] * r)
        h = (h - n) * z + n
        out.append(h)
        gates.append(torch.cat([r, z, n, gh[:, 2 * D:]], 1))
    return torch.stack(out, 1), torch.stack(gates, 1)


# row layouts (gru_xcd.hip gx_layout): B = 128 one 16-row tile per group; B <= 64 fewer valid
# rows per tile on all 8 XCDs; 256 / 300 / 512 several tiles per group (configs[3]'s 512 rows on
# one GPU, 256 on two); 600 two launches (512 + 88 rows); D = 512 / 256 other group widths
XCD_SHAPES = [(128, 1024, 64), (64, 1024, 5), (100, 256, 9), (16, 512, 3), (512, 1024, 16),
              (256, 1024, 9), (300, 1024, 5), (600, 1024, 4), (64, 1024, 64), (512, 512, 7)]


@pytest.mark.parametrize('B,D,Fr', XCD_SHAPES)
def test_gru_xcd_fwd(hip, B, D, Fr):
    """XCD-grouped persistent GRU forward (gru_xcd.hip) vs the torch recurrence; same outputs
    as the gru_seq kernel within MFMA summation-order noise."""
    T = torch.bfloat16
    nb = hip.gru_xcd_work_bytes(T, B, D)
    if not nb:
        pytest.skip('gru_xcd not supported on this device')
    g = torch.Generator().manual_seed(B + D + 1)
    whh = (torch.randn(3 * D, D, generator=g) * 0.03).to(DEV, T)
    bhh = (torch.randn(3 * D, generator=g) * 0.1).to(DEV)
    gi = (torch.randn(B * Fr, 3 * D, generator=g) * 0.5).to(DEV)
    h0 = (torch.randn(B, D, generator=g) * 0.5).to(DEV)
    out = torch.full((B, Fr, D), float('nan'), device=DEV)
    outT = torch.zeros((B, Fr, D), device=DEV, dtype=T)
    gt = torch.full((B, Fr, 4 * D), float('nan'), device=DEV)
    work = torch.full((nb,), 7, device=DEV, dtype=torch.uint8)
    hip.lib().call('srnn_gru_xcd_fwd', hip.BF16, B, D, Fr, hip.ptr(gi), Fr * 3 * D, 3 * D,
                   hip.ptr(h0), hip.ptr(whh), hip.ptr(bhh), hip.ptr(out), hip.ptr(outT), Fr * D,
                   D, hip.ptr(gt), Fr * 4 * D, 4 * D, hip.ptr(work), nb, hip.stream())
    torch.cuda.synchronize()
    assert hip.lib().dll.srnn_gru_xcd_error(hip.ptr(work)) == 0, 'gru_xcd gave up waiting'
    ref_out, ref_gt = _gru_ref(gi.cpu(), h0.cpu(), whh.cpu(), bhh.cpu(), Fr)
    torch.testing.assert_close(out.cpu(), ref_out, atol=2e-3, rtol=0)
    torch.testing.assert_close(gt.cpu(), ref_gt, atol=2e-3, rtol=0)
    torch.testing.assert_close(outT.float().cpu(), out.cpu().to(T).float(), atol=0, rtol=0)
    # srnn_gru_xcd_fwd2: the same outputs bit for bit, plus [bf16(h0), outT[:, :F-1]]
    out2 = torch.full_like(out, float('nan'))
    outT2 = torch.zeros_like(outT)
    gt2 = torch.full_like(gt, float('nan'))
    hp = torch.full((B, Fr, D), float('nan'), device=DEV).to(T)
    work.fill_(7)
    hip.lib().call('srnn_gru_xcd_fwd2', hip.BF16, B, D, Fr, hip.ptr(gi), Fr * 3 * D, 3 * D,
                   hip.ptr(h0), hip.ptr(whh), hip.ptr(bhh), hip.ptr(out2), hip.ptr(outT2), Fr * D,
                   D, hip.ptr(gt2), Fr * 4 * D, 4 * D, hip.ptr(hp), hip.ptr(work), nb,
                   hip.stream())
    torch.cuda.synchronize()
    assert hip.lib().dll.srnn_gru_xcd_error(hip.ptr(work)) == 0, 'gru_xcd gave up waiting'
    assert torch.equal(out2, out) and torch.equal(outT2, outT) and torch.equal(gt2, gt)
    assert torch.equal(hp[:, 0], h0.to(T))
    assert torch.equal(hp[:, 1:], outT[:, :-1])


@pytest.mark.parametrize('B,D,Fr', XCD_SHAPES)
def test_gru_xcd_bwd(hip, B, D, Fr):
    """XCD-grouped persistent GRU backward vs torch autograd of the same recurrence (bf16
    W_hh and bf16 dgh operands on the MFMA path: tolerance, not bits)."""
    T = torch.bfloat16
    nb = hip.gru_xcd_bwd_work_bytes(T, B, D)
    if not nb:
        pytest.skip('gru_xcd not supported on this device')
    g = torch.Generator().manual_seed(B * 7 + D)
    whh = (torch.randn(3 * D, D, generator=g) * 0.03).to(T)
    bhh = torch.randn(3 * D, generator=g) * 0.1
    gi = torch.randn(B * Fr, 3 * D, generator=g) * 0.5
    h0 = torch.randn(B, D, generator=g) * 0.5
    dy = torch.randn(B, Fr, D, generator=g) * 0.1
    # forward (fp32, with the saved gates the kernel consumes)
    out, gates = _gru_ref(gi, h0, whh, bhh, Fr)
    # reference backward: autograd through the fp32 recurrence with fp32 weights
    W = whh.float().requires_grad_(False)
    gi_r = gi.clone().requires_grad_(True)
    h0_r = h0.clone().requires_grad_(True)
    h = h0_r
    outs = []
    for t in range(Fr):
        gh = h @ W.t() + bhh
        gg = gi_r.reshape(B, Fr, 3 * D)[:, t]
        r = torch.sigmoid(gh[:, :D] + gg[:, :D])
        z = torch.sigmoid(gh[:, D:2 * D] + gg[:, D:2 * D])
        n = torch.tanh(gg[:, 2 * D:] + gh[:, 2 * D:] * r)
        h = (h - n) * z + n
        outs.append(h)
    torch.autograd.backward(torch.stack(outs, 1), dy)
    whh_t = whh.float().t().contiguous().to(DEV, T)
    dgh = torch.full((B, Fr, 3 * D), float('nan'), device=DEV)
    dgh_lp = torch.zeros((B, Fr, 3 * D), device=DEV, dtype=T)
    dgi = torch.full((B, Fr, 3 * D), float('nan'), device=DEV)
    ddir0 = torch.full((B, D), float('nan'), device=DEV)
    work = torch.full((nb,), 7, device=DEV, dtype=torch.uint8)
    dyd, gtd, outd, h0d = dy.to(DEV), gates.to(DEV), out.to(DEV), h0.to(DEV)
    hip.lib().call('srnn_gru_xcd_bwd', hip.BF16, B, D, Fr, hip.ptr(dyd), Fr * D, D, hip.ptr(gtd),
                   Fr * 4 * D, 4 * D, hip.ptr(outd), Fr * D, D, hip.ptr(h0d), hip.ptr(whh_t),
                   hip.ptr(dgh), hip.ptr(dgh_lp), hip.ptr(dgi), Fr * 3 * D, 3 * D,
                   hip.ptr(ddir0), hip.ptr(work), nb, hip.stream())
    torch.cuda.synchronize()
    assert hip.lib().dll.srnn_gru_xcd_error(hip.ptr(work)) == 0, 'gru_xcd_bwd gave up waiting'
    # dgi = dL/d(gi): exactly the reference's input-projection gradient
    ref_dgi = gi_r.grad.reshape(B, Fr, 3 * D)
    scale = ref_dgi.abs().max().item()
    torch.testing.assert_close(dgi.cpu(), ref_dgi, atol=2e-2 * scale, rtol=0)
    # dh_0 = dgh_0 . W_hh + ddir0
    dh0 = dgh[:, 0].cpu() @ whh.float() + ddir0.cpu()
    torch.testing.assert_close(dh0, h0_r.grad, atol=2e-2 * h0_r.grad.abs().max().item(), rtol=0)
    torch.testing.assert_close(dgh_lp.float().cpu(), dgh.cpu().to(T).float(), atol=0, rtol=0)
    # srnn_gru_xcd_bwd2 (the training path): the same dgh / dgi in bf16 bit for bit, and the
    # per-row bias-gradient sums over t of [dar | daz | dghn | dan]
    dgh2 = torch.zeros((B, Fr, 3 * D), device=DEV, dtype=T)
    dgi2 = torch.zeros((B, Fr, 3 * D), device=DEV, dtype=T)
    bsum = torch.full((B, 4 * D), float('nan'), device=DEV)
    ddir2 = torch.full((B, D), float('nan'), device=DEV)
    work.fill_(7)
    hip.lib().call('srnn_gru_xcd_bwd2', hip.BF16, B, D, Fr, hip.ptr(dyd), Fr * D, D, hip.ptr(gtd),
                   Fr * 4 * D, 4 * D, hip.ptr(outd), Fr * D, D, hip.ptr(h0d), hip.ptr(whh_t),
                   None, hip.ptr(dgh2), None, hip.ptr(dgi2), hip.ptr(bsum), Fr * 3 * D, 3 * D,
                   hip.ptr(ddir2), hip.ptr(work), nb, hip.stream())
    torch.cuda.synchronize()
    assert hip.lib().dll.srnn_gru_xcd_error(hip.ptr(work)) == 0, 'gru_xcd_bwd2 gave up waiting'
    assert torch.equal(dgh2, dgh_lp) and torch.equal(ddir2, ddir0)
    assert torch.equal(dgi2, dgi.to(T))
    ref_bs = torch.cat([dgh.sum(1), dgi[:, :, 2 * D:].sum(1)], 1)
    torch.testing.assert_close(bsum, ref_bs, atol=1e-5 * ref_bs.abs().max().item(), rtol=1e-5)


@pytest.mark.parametrize('D', [1024, 512])
def test_gru_xcd_layouts_bit_identical(hip, D):
    """Rows are independent and every row's arithmetic is the same in every row layout, so a
    512-row sweep (4 tiles per group), a 64-row one (8 valid rows per tile), 600 rows (two
    launches) and the 128-row launches of the same rows give identical bits, forward and
    backward (a size-independent check of the B > 128 layouts against the B = 128 one)."""
    T = torch.bfloat16
    Fr = 6
    g = torch.Generator().manual_seed(D + 5)
    Bt = 600
    whh = (torch.randn(3 * D, D, generator=g) * 0.03).to(DEV, T)
    whh_t = whh.float().t().contiguous().to(T)
    bhh = (torch.randn(3 * D, generator=g) * 0.1).to(DEV)
    gi = (torch.randn(Bt, Fr, 3 * D, generator=g) * 0.5).to(DEV)
    h0 = (torch.randn(Bt, D, generator=g) * 0.5).to(DEV)
    dy = (torch.randn(Bt, Fr, D, generator=g) * 0.1).to(DEV)

    def run(r0, n):
        nf = hip.gru_xcd_work_bytes(T, n, D)
        nb = hip.gru_xcd_bwd_work_bytes(T, n, D)
        assert nf and nb
        wf = torch.empty(nf, device=DEV, dtype=torch.uint8)
        wb = torch.empty(nb, device=DEV, dtype=torch.uint8)
        out = torch.empty((n, Fr, D), device=DEV)
        outT = torch.empty((n, Fr, D), device=DEV, dtype=T)
        gt = torch.empty((n, Fr, 4 * D), device=DEV)
        hp = torch.empty((n, Fr, D), device=DEV, dtype=T)
        gi_ = gi[r0:r0 + n].contiguous()
        h0_ = h0[r0:r0 + n].contiguous()
        hip.lib().call('srnn_gru_xcd_fwd2', hip.BF16, n, D, Fr, hip.ptr(gi_), Fr * 3 * D, 3 * D,
                       hip.ptr(h0_), hip.ptr(whh), hip.ptr(bhh), hip.ptr(out), hip.ptr(outT),
                       Fr * D, D, hip.ptr(gt), Fr * 4 * D, 4 * D, hip.ptr(hp), hip.ptr(wf), nf,
                       hip.stream())
        dgh = torch.empty((n, Fr, 3 * D), device=DEV, dtype=T)
        dgi = torch.empty((n, Fr, 3 * D), device=DEV, dtype=T)
        bsum = torch.empty((n, 4 * D), device=DEV)
        ddir = torch.empty((n, D), device=DEV)
        dy_ = dy[r0:r0 + n].contiguous()
        hip.lib().call('srnn_gru_xcd_bwd2', hip.BF16, n, D, Fr, hip.ptr(dy_), Fr * D, D,
                       hip.ptr(gt), Fr * 4 * D, 4 * D, hip.ptr(out), Fr * D, D, hip.ptr(h0_),
                       hip.ptr(whh_t), None, hip.ptr(dgh), None, hip.ptr(dgi), hip.ptr(bsum),
                       Fr * 3 * D, 3 * D, hip.ptr(ddir), hip.ptr(wb), nb, hip.stream())
        torch.cuda.synchronize()
        assert hip.lib().dll.srnn_gru_xcd_error(hip.ptr(wf)) == 0
        assert hip.lib().dll.srnn_gru_xcd_error(hip.ptr(wb)) == 0
        return [x.cpu() for x in (out, outT, gt, hp, dgh, dgi, bsum, ddir)]

    ref = [run(r0, 128) for r0 in range(0, 512, 128)] + [run(512, 88)]
    ref = [torch.cat([c[i] for c in ref], 0) for i in range(8)]
    for r0, n in ((0, 512), (0, 600), (64, 64), (0, 256), (128, 300)):
        got = run(r0, n)
        for i, (a, b) in enumerate(zip(got, ref)):
            assert torch.equal(a, b[r0:r0 + n]), (r0, n, i)


@pytest.mark.parametrize('B', [512, 256, 128])
def test_gru_xcd_fwd_compile_time_d_bit_identical(hip, B, monkeypatch):
    """The D = 1024 forward instantiations (D at compile time, gru_xcd_fwd_kernel<4, MT,
    1024>, the training path's) give the runtime-D kernel's bits at every tile count."""
    T = torch.bfloat16
    D, Fr = 1024, 7
    g = torch.Generator().manual_seed(B + 11)
    whh = (torch.randn(3 * D, D, generator=g) * 0.03).to(DEV, T)
    bhh = (torch.randn(3 * D, generator=g) * 0.1).to(DEV)
    gi = (torch.randn(B, Fr, 3 * D, generator=g) * 0.5).to(DEV)
    h0 = (torch.randn(B, D, generator=g) * 0.5).to(DEV)
    nf = hip.gru_xcd_work_bytes(T, B, D)
    outs = []
    for dc in ('1', '0'):
        monkeypatch.setenv('SRNN_GX_DC', dc)
        wf = torch.empty(nf, device=DEV, dtype=torch.uint8)
        out = torch.empty((B, Fr, D), device=DEV)
        outT = torch.empty((B, Fr, D), device=DEV, dtype=T)
        gt = torch.empty((B, Fr, 4 * D), device=DEV)
        hp = torch.empty((B, Fr, D), device=DEV, dtype=T)
        hip.lib().call('srnn_gru_xcd_fwd2', hip.BF16, B, D, Fr, hip.ptr(gi), Fr * 3 * D, 3 * D,
                       hip.ptr(h0), hip.ptr(whh), hip.ptr(bhh), hip.ptr(out), hip.ptr(outT),
                       Fr * D, D, hip.ptr(gt), Fr * 4 * D, 4 * D, hip.ptr(hp), hip.ptr(wf), nf,
                       hip.stream())
        torch.cuda.synchronize()
        assert hip.lib().dll.srnn_gru_xcd_error(hip.ptr(wf)) == 0
        outs.append([x.cpu() for x in (out, outT, gt, hp)])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize('B,D,Fr', [(128, 1024, 16), (64, 1024, 5), (100, 256, 9)])
def test_gru_seq_bwd_matches_steps(hip, B, D, Fr):
    """Persistent whole-sequence GRU backward == Fr per-step backward launches, bit for bit."""
    T = torch.bfloat16
    if not hip.gru_seq_supported(T, B, D):
        pytest.skip('persistent GRU not supported on this device')
    g = torch.Generator().manual_seed(B * 7 + D)
    whh = (torch.randn(3 * D, D, generator=g) * 0.03).to(DEV, T)
    whhT = whh.t().contiguous()
    # forward state from a real recurrence (per-step cells)
    bhh = (torch.randn(3 * D, generator=g) * 0.1).to(DEV)
    gi = (torch.randn(B * Fr, 3 * D, generator=g) * 0.5).to(DEV)
    h0 = (torch.randn(B, D, generator=g) * 0.5).to(DEV)
    h0T = h0.to(T)
    out = torch.empty(B, Fr, D, device=DEV)
    outT = torch.empty(B, Fr, D, device=DEV, dtype=T)
    gt = torch.empty(B, Fr, 4 * D, device=DEV)
    for t in range(Fr):
        hp_t, hp_f, ldh = (h0T, h0, D) if t == 0 else (outT[:, t - 1], out[:, t - 1], Fr * D)
        hip.lib().call('srnn_gru_cell', hip.BF16, B, D, D, None, 0, None, None, hip.ptr(gi[t:]),
                       Fr * 3 * D, hip.ptr(hp_t), ldh, hip.ptr(hp_f), ldh, hip.ptr(whh),
                       hip.ptr(bhh), hip.ptr(out[:, t]), Fr * D, hip.ptr(outT[:, t]), Fr * D,
                       hip.ptr(gt[:, t]), Fr * 4 * D, hip.stream())
    dy = (torch.randn(B, Fr, D, generator=g) * 0.1).to(DEV)
    res = {}
    for mode in ('seq', 'steps'):
        dgh = torch.full((B, Fr, 3 * D), float('nan'), device=DEV)
        dghT = torch.zeros((B, Fr, 3 * D), device=DEV, dtype=T)
        dgi = torch.full((B, Fr, 3 * D), float('nan'), device=DEV)
        ddir = [torch.zeros(B, D, device=DEV) for _ in range(2)]
        if mode == 'seq':
            nw = 64 * ((B + 31) // 32) + 1
            work = torch.full((nw,), 7, device=DEV, dtype=torch.int32)
            hip.lib().call('srnn_gru_seq_bwd', hip.BF16, B, D, Fr, hip.ptr(dy), Fr * D, D,
                           hip.ptr(gt), Fr * 4 * D, 4 * D, hip.ptr(out), Fr * D, D, hip.ptr(h0),
                           hip.ptr(whhT), hip.ptr(dgh), hip.ptr(dghT), hip.ptr(dgi), Fr * 3 * D,
                           3 * D, hip.ptr(ddir[0]), hip.ptr(work), nw * 4, hip.stream())
            torch.cuda.synchronize()
            assert int(work[nw - 1]) == 0, 'persistent GRU backward gave up waiting'
        else:
            for t in reversed(range(Fr)):
                nxt = t + 1 < Fr
                hp, ldhp = (out[:, t - 1], Fr * D) if t > 0 else (h0, D)
                hip.lib().call('srnn_gru_cell_bwd', hip.BF16, B, D, hip.ptr(dy[:, t]), Fr * D,
                               hip.ptr(dghT[:, t + 1]) if nxt else None, Fr * 3 * D,
                               hip.ptr(ddir[(t + 1) % 2]) if nxt else None, hip.ptr(whh),
                               hip.ptr(whhT), hip.ptr(gt[:, t]), Fr * 4 * D, hip.ptr(hp), ldhp,
                               hip.ptr(dgh[:, t]), Fr * 3 * D, hip.ptr(dghT[:, t]), Fr * 3 * D,
                               hip.ptr(dgi[:, t]), Fr * 3 * D, hip.ptr(ddir[t % 2]),
                               hip.stream())
        res[mode] = (dgh.cpu(), dghT.float().cpu(), dgi.cpu(), ddir[0].cpu())
    for name, a, b in zip(('dgh', 'dgh_lp', 'dgi', 'ddir0'), res['seq'], res['steps']):
        bad = (a != b).nonzero()
        assert bad.numel() == 0, (name, bad.shape[0], bad[:4].tolist(),
                                  (a - b).abs().max().item())


def test_segsum(hip):
    B, F, D = 7, 16, 1030
    x = _rand(B * F, D + 3, seed=9).to(DEV)
    out = torch.empty(B, D, device=DEV)
    hip.lib().call('srnn_segsum', hip.ptr(x), D + 3, B, F, D, hip.ptr(out), hip.stream())
    ref = x[:, :D].reshape(B, F, D).sum(1)
    torch.testing.assert_close(out, ref, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('M,N,K', [(128, 1024, 1024), (67, 256, 512), (128, 40, 256),
                                   (256, 2048, 256), (128, 16384, 1024), (100, 4096, 1024),
                                   (65, 16448, 256), (128, 19456, 1024), (120, 20480, 256),
                                   (128, 12288, 1024)])
def test_gemm_skinny_ring(hip, dtype, M, N, K):
    """Skinny NT deep-ring kernel (tile 4 forces it), with the full epilogue; N = 19456 and
    20480 take the 80-wide tiles (the generation tick's [W_up; W_hh] GEMM), 12288 the 48-wide."""
    A, W = _rand(M, K, seed=1), _rand(N, K, seed=2)
    bias, cin, mask = _rand(N, seed=3), _rand(M, N, seed=4), _rand(M, N, seed=5)
    Ad, Wd = A.to(DEV, dtype), W.to(DEV, dtype)
    out = hip.gemm(Ad, Wd, transB=True, bias=bias.to(DEV), cin=cin.to(DEV), beta=0.25,
                   relu=True, mask=mask.to(DEV, dtype), tile=4)
    ref = ((Ad.float().cpu() @ Wd.float().cpu().t()) + 0.25 * cin + bias).clamp_min(0)
    ref = ref * (mask.to(dtype).float() > 0)
    tol = 1e-4 * np.sqrt(K) if dtype == torch.float32 else 2e-3 * np.sqrt(K)
    torch.testing.assert_close(out.cpu(), ref, atol=tol, rtol=1e-4)


def test_gemm_bf16_out_batched_mask(hip):
    Bt, M, N, K = 3, 40, 72, 48
    A = _rand(Bt, M, K, seed=5).to(DEV)
    W = _rand(Bt, N, K, seed=6).to(DEV)
    mask = _rand(Bt, M, N, seed=7).to(DEV)
    out = torch.empty(Bt, M, N, device=DEV, dtype=torch.bfloat16)
    hip.gemm(A[0], W[0], transB=True, out=out[0], M=M, N=N, K=K, lda=K, ldb=K, ldc=N, batch=Bt,
             sA=M * K, sB=N * K, sC=M * N, mask=mask[0])
    ref = torch.bmm(A.cpu(), W.cpu().transpose(1, 2)) * (mask.cpu() > 0)
    torch.testing.assert_close(out.float().cpu(), ref, atol=2e-2, rtol=1e-2)


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('with_x', [False, True])
@pytest.mark.parametrize('D', [80, 256, 1024])   # 256, 1024: deep-ring kernel path
def test_gru_cell(hip, dtype, with_x, D):
    B = 67
    x = _rand(B, D, seed=1).to(DEV)
    h = _rand(B, D, seed=2).to(DEV)
    wih = _rand(3 * D, D, scale=0.3, seed=3).to(DEV)
    whh = _rand(3 * D, D, scale=0.3, seed=4).to(DEV)
    bih = _rand(3 * D, scale=0.1, seed=5).to(DEV)
    bhh = _rand(3 * D, scale=0.1, seed=6).to(DEV)
    xT, hT, wihT, whhT = (t.to(dtype) for t in (x, h, wih, whh))
    gi = hip.linear(xT, wihT, bias=bih)
    hout = torch.empty(B, D, device=DEV)
    gates = torch.empty(B, 4 * D, device=DEV)
    hip.lib().call('srnn_gru_cell', hip.dcode(dtype), B, D, D,
                   hip.ptr(xT) if with_x else None, D, hip.ptr(wihT), hip.ptr(bih),
                   None if with_x else hip.ptr(gi), 3 * D, hip.ptr(hT), D, hip.ptr(h), D,
                   hip.ptr(whhT), hip.ptr(bhh), hip.ptr(hout), D, None, 0, hip.ptr(gates), 4 * D,
                   hip.stream())
    xf, hf = xT.float().cpu(), hT.float().cpu()
    gi_r = xf @ wihT.float().cpu().t() + bih.cpu()
    gh_r = hf @ whhT.float().cpu().t() + bhh.cpu()
    r = torch.sigmoid(gi_r[:, :D] + gh_r[:, :D])
    z = torch.sigmoid(gi_r[:, D:2 * D] + gh_r[:, D:2 * D])
    n = torch.tanh(gi_r[:, 2 * D:] + r * gh_r[:, 2 * D:])
    ref = (h.cpu() - n) * z + n
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    torch.testing.assert_close(hout.cpu(), ref, atol=tol, rtol=0)
    torch.testing.assert_close(gates[:, 3 * D:].cpu(), gh_r[:, 2 * D:], atol=tol * 10, rtol=0)


@pytest.mark.parametrize('D,ring', [(48, False), (256, True)])
def test_gru_cell_bwd(hip, D, ring):
    """Gate backward + dgh . W_hh against autograd of the torch formula (fp32)."""
    B = 33
    h = _rand(B, D, seed=2).requires_grad_(True)
    gi = _rand(B, 3 * D, seed=3)
    whh = _rand(3 * D, D, scale=0.3, seed=4)
    bhh = _rand(3 * D, scale=0.1, seed=6)
    gh = h @ whh.t() + bhh
    r = torch.sigmoid(gi[:, :D] + gh[:, :D])
    z = torch.sigmoid(gi[:, D:2 * D] + gh[:, D:2 * D])
    n = torch.tanh(gi[:, 2 * D:] + r * gh[:, 2 * D:])
    hn = (h - n) * z + n
    dy = _rand(B, D, seed=9)
    gh.retain_grad()
    hn.backward(dy)
    gates = torch.cat([r, z, n, gh[:, 2 * D:]], 1).detach().to(DEV)
    dgh = torch.empty(B, 3 * D, device=DEV)
    dgi = torch.empty(B, 3 * D, device=DEV)
    ddir = torch.empty(B, D, device=DEV)
    hd = h.detach().to(DEV)
    dyd = dy.to(DEV)
    hip.lib().call('srnn_gru_cell_bwd', hip.F32, B, D, hip.ptr(dyd), D, None, 0, None,
                   hip.ptr(whh.to(DEV)), None, hip.ptr(gates), 4 * D, hip.ptr(hd), D, hip.ptr(dgh),
                   3 * D, None, 0, hip.ptr(dgi), 3 * D, hip.ptr(ddir), hip.stream())
    torch.testing.assert_close(dgh.cpu(), gh.grad, atol=1e-5, rtol=1e-4)
    # a second step consuming dgh as dgh_next exercises the dgh . W_hh product (ring path
    # when W_hh^T is given)
    whh_d = whh.to(DEV)
    whh_t = whh_d.t().contiguous() if ring else None
    dgh2 = torch.empty_like(dgh)
    dgi2 = torch.empty_like(dgi)
    ddir2 = torch.empty_like(ddir)
    hip.lib().call('srnn_gru_cell_bwd', hip.F32, B, D, hip.ptr(dyd), D, hip.ptr(dgh), 3 * D,
                   hip.ptr(ddir), hip.ptr(whh_d), hip.ptr(whh_t), hip.ptr(gates), 4 * D,
                   hip.ptr(hd), D, hip.ptr(dgh2), 3 * D, None, 0, hip.ptr(dgi2), 3 * D,
                   hip.ptr(ddir2), hip.stream())
    dh2 = dy + ddir.cpu() + dgh.cpu() @ whh
    g = gates.cpu()
    r_, z_, n_, ghn_ = g[:, :D], g[:, D:2 * D], g[:, 2 * D:3 * D], g[:, 3 * D:]
    dan = dh2 * (1 - z_) * (1 - n_ * n_)
    ref_dgh2 = torch.cat([dan * ghn_ * r_ * (1 - r_), dh2 * (h.detach() - n_) * z_ * (1 - z_),
                          dan * r_], 1)
    torch.testing.assert_close(dgh2.cpu(), ref_dgh2, atol=2e-5, rtol=1e-4)
    torch.testing.assert_close(ddir2.cpu(), dh2 * z_, atol=2e-5, rtol=1e-4)
    # dh_prev = z*dy + dgh . W_hh  ==  autograd's h.grad
    dh = hip.gemm(dgh, whh.to(DEV), cin=ddir, beta=1.0)
    torch.testing.assert_close(dh.cpu(), h.grad, atol=1e-5, rtol=1e-4)


def test_uquantize_f32_exhaustive(hip):
    """Every float32 in [-1, 1] (2.13e9 values) against the reference staircase."""
    g = golden('ulaw')
    steps = torch.from_numpy(g['f32_steps_x']).to(DEV)
    one = 0x3F800000
    CH = 1 << 27
    for sign in (0, 1):
        for lo in range(0, one + 1, CH):
            hi = min(one, lo + CH - 1)
            bits = torch.arange(lo, hi + 1, device=DEV, dtype=torch.int32)
            x = bits.view(torch.float32)
            if sign:
                x = -x        # exact: flips the sign bit
            q = torch.empty(x.numel(), device=DEV, dtype=torch.long)
            hip.lib().call('srnn_uquantize_f32', hip.ptr(x), hip.ptr(q), x.numel(), 256,
                           hip.stream())
            ref = torch.searchsorted(steps, x, right=True)
            assert torch.equal(q, ref), 'mismatch in chunk %x' % lo


@pytest.mark.parametrize('mode', [0, 1])
def test_udequantize_window_in_place(hip, mode):
    """srnn_udequantize2d on a strided window of the index stream (Predictor's per-tier
    slices) equals srnn_udequantize of the copied slice, bit for bit."""
    import utils
    g = torch.Generator().manual_seed(11)
    seq = torch.randint(0, 256, (5, 300), generator=g).to(DEV)
    win = seq[:, 37:37 + 211]
    assert not win.is_contiguous()
    got = utils._dequant(win, 256, 2.0, mode)
    want = utils._dequant(win.contiguous(), 256, 2.0, mode)
    assert torch.equal(got, want)


def test_uquantize_kats(hip):
    g = golden('ulaw')
    import utils
    for k in ('32', '64'):
        x = torch.from_numpy(g['kat_x' + k]).to(DEV)
        assert np.array_equal(utils.uquantize(x, 256).cpu().numpy(), g['kat_q' + k])
    lut = utils.udequantize(torch.arange(256, device=DEV), 256).cpu().numpy()
    assert np.array_equal(lut, g['lut'])
    # linear dequantize
    lin = utils.linear_dequantize(torch.arange(256, device=DEV), 256).cpu().numpy()
    assert np.array_equal(lin, g['lin_lut'])


def test_logsoftmax_and_sampler(hip):
    R, Q = 37, 256
    z = (_rand(R, Q, seed=11) * 6).to(DEV)
    logp = torch.empty(R, Q, device=DEV)
    hip.lib().call('srnn_logsoftmax_nll', hip.ptr(z), Q, None, 0, 1, R, Q, None, hip.ptr(logp), Q,
                   None, hip.F32, 0, 0.0, hip.stream())
    torch.testing.assert_close(logp.cpu(), torch.log_softmax(z.cpu(), 1), atol=2e-6, rtol=0)


@pytest.mark.parametrize('dtype,udtype', [(torch.float32, torch.float32),
                                          (torch.bfloat16, torch.float32),
                                          (torch.bfloat16, torch.bfloat16)])
@pytest.mark.parametrize('B,Tl,D,FS0,Q', [(2, 40, 72, 16, 256), (8, 1024, 256, 16, 256),
                                          (5, 1000, 384, 20, 64), (4, 2048, 1024, 16, 256)])
def test_mlp_l1_gather(hip, dtype, udtype, B, Tl, D, FS0, Q):
    """a1 = relu(upper + sum_k Tab[k][x_{t+k}]) -- both the generic and the XCD-sliced
    (rows >= 4096, D % 128 == 0) kernels."""
    g = torch.Generator().manual_seed(Tl + D)
    tab = _rand(FS0, Q, D, seed=D).to(dtype)
    x = torch.randint(0, Q, (B, Tl + FS0 - 1), generator=g)
    upper = _rand(B * Tl, D, seed=5).to(udtype)
    idx = torch.stack([x[:, k:k + Tl] for k in range(FS0)], -1).reshape(B * Tl, FS0)
    ref = upper.float().clone()
    tf = tab.float()
    for k in range(FS0):
        ref += tf[k][idx[:, k]]
    ref = ref.clamp_min(0)
    out = torch.empty(B * Tl, D, device=DEV, dtype=dtype)
    tab_d, x_d, up_d = tab.to(DEV), x.to(DEV), upper.to(DEV)     # keep alive over the call
    hip.lib().call('srnn_mlp_l1', hip.dcode(dtype), hip.ptr(tab_d), hip.ptr(x_d), x.shape[1], 0,
                   B, Tl, hip.dcode(udtype), hip.ptr(up_d), D, hip.ptr(out), D, D, FS0, Q,
                   hip.stream())
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    torch.testing.assert_close(out.float().cpu(), ref, atol=tol, rtol=tol)


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('B,Tl,D,FS0,Q', [(3, 37, 72, 16, 256), (5, 64, 1024, 16, 256),
                                          (2, 50, 40, 20, 256), (4, 30, 33, 4, 64), (0, 8, 16, 16, 256)])
def test_mlp_dtab_scatter(hip, dtype, B, Tl, D, FS0, Q):
    """dTab[q][k][:] = sum over (b, t) with x[b, t + k] == q of da[b, t, :] -- the
    embedding . conv backward (model.py:274-285).  Fixed-point accumulation: within 2^-40
    per term of the fp64 sum, and bit-identical from run to run."""
    g = torch.Generator().manual_seed(B * 1000 + D)
    x = torch.randint(0, Q, (max(B, 1), Tl + FS0 - 1 + 3), generator=g)[:B]
    x[:, 5:12] = 7                                  # runs of equal indices (silence)
    da = (_rand(max(B, 1) * Tl, D, scale=1e-3, seed=D)[:B * Tl]).to(dtype)
    ref = torch.zeros(Q, FS0, D, dtype=torch.float64)
    for k in range(FS0):
        ref[:, k].index_add_(0, x[:, k:k + Tl].reshape(-1), da.double())
    work = torch.empty(Q * FS0 * D, device=DEV, dtype=torch.int64)
    outs = []
    for _ in range(2):
        out = torch.empty(Q, FS0, D, device=DEV, dtype=torch.float32)
        xd, dad = x.to(DEV).contiguous(), da.to(DEV).contiguous()
        hip.lib().call('srnn_mlp_dtab', hip.dcode(dtype), hip.ptr(dad), D, hip.ptr(xd), x.shape[1],
                       0, B, Tl, hip.ptr(out), hip.F32, D, FS0, Q, hip.ptr(work), work.numel() * 8,
                       hip.stream())
        outs.append(out.cpu())
    assert torch.equal(outs[0], outs[1])
    torch.testing.assert_close(outs[0].double(), ref, atol=1e-9 + 1e-12 * B * Tl, rtol=1e-6)


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('B,Tl,D', [(5, 64, 1024), (128, 1024, 1024), (3, 37, 72), (2, 100, 768)])
def test_mlp_dtab2_colsum(hip, dtype, B, Tl, D):
    """srnn_mlp_dtab2: the same dTab as srnn_mlp_dtab, plus (direct path, D >= 768) the
    residue column sums colsum[j * D + c] = sum_{b, t = j mod 16} da[b, t, c]."""
    import ctypes
    FS0, Q = 16, 256
    g = torch.Generator().manual_seed(B + Tl + D)
    x = torch.randint(0, Q, (B, Tl + FS0 - 1), generator=g).to(DEV)
    da = (torch.randn(B * Tl, D, generator=g) * 1e-3).to(DEV, dtype)
    work = torch.empty(Q * FS0 * D, device=DEV, dtype=torch.int64)
    ref_tab = torch.empty(Q, FS0, D, device=DEV)
    hip.lib().call('srnn_mlp_dtab', hip.dcode(dtype), hip.ptr(da), D, hip.ptr(x), x.shape[1], 0, B,
                   Tl, hip.ptr(ref_tab), hip.F32, D, FS0, Q, hip.ptr(work), work.numel() * 8,
                   hip.stream())
    tab = torch.empty(Q, FS0, D, device=DEV)
    colsum = torch.full((FS0 * D,), float('nan'), device=DEV)
    done = ctypes.c_int(-1)
    hip.lib().call('srnn_mlp_dtab2', hip.dcode(dtype), hip.ptr(da), D, hip.ptr(x), x.shape[1], 0,
                   B, Tl, hip.ptr(tab), hip.F32, D, FS0, Q, hip.ptr(work), work.numel() * 8,
                   hip.ptr(colsum), ctypes.byref(done), hip.stream())
    torch.cuda.synchronize()
    assert torch.equal(tab, ref_tab)
    assert done.value == (1 if D >= 768 else 0)
    if done.value:
        ref = da.double().reshape(B, Tl, D)
        pad = (-Tl) % FS0
        ref = torch.cat([ref, ref.new_zeros(B, pad, D)], 1).reshape(B, -1, FS0, D).sum((0, 1))
        torch.testing.assert_close(colsum.double().reshape(FS0, D), ref, atol=1e-9, rtol=1e-6)


@pytest.mark.parametrize('B,Tl,skew', [(128, 1024, False), (9, 1024, True), (64, 256, True),
                                        (3, 37, False), (5, 70, False), (2, 115, True)])
def test_mlp_dtab_packed_bf16(hip, monkeypatch, B, Tl, skew):
    """The packed two-columns-per-atomic dTab (bf16 in / out, dtab_pk_kernel) against the exact
    2^-40 path and an fp64 scatter.  Its scale comes from max |da| and the most frequent sample
    value (skew: 60 % of the positions hold one value, the bound's worst case), so every sum
    is exact to 2^-30 of amax x count: the bf16 outputs equal the exact path's or differ by
    one bf16 rounding step; every entry is within count_max / (2 S) of the fp64 sum (plus its
    bf16 rounding); the column sums are identical."""
    import ctypes
    FS0, Q, D = 16, 256, 1024
    g = torch.Generator().manual_seed(B * 7 + Tl)
    x = torch.randint(0, Q, (B, Tl + FS0 - 1), generator=g)
    if skew:
        x[torch.rand(x.shape, generator=g) < 0.6] = 128
    x = x.to(DEV)
    da = (torch.randn(B * Tl, D, generator=g) * 1e-4).to(DEV, torch.bfloat16)
    da[7] *= 50                                       # one large row sets amax
    work = torch.empty(Q * FS0 * D, device=DEV, dtype=torch.int64)

    def run(pack):
        monkeypatch.setenv('SRNN_DTAB_PACK', '1' if pack else '0')
        tab = torch.empty(Q, FS0, D, device=DEV, dtype=torch.bfloat16)
        colsum = torch.full((FS0 * D,), float('nan'), device=DEV)
        done = ctypes.c_int(-1)
        hip.lib().call('srnn_mlp_dtab2', hip.BF16, hip.ptr(da), D, hip.ptr(x), x.shape[1], 0,
                       B, Tl, hip.ptr(tab), hip.BF16, D, FS0, Q, hip.ptr(work),
                       work.numel() * 8, hip.ptr(colsum), ctypes.byref(done), hip.stream())
        torch.cuda.synchronize()
        assert done.value == 1
        return tab.float().cpu(), colsum.cpu()

    t_exact, c_exact = run(False)
    t_pk, c_pk = run(True)
    t_pk2, _ = run(True)
    assert torch.equal(t_pk, t_pk2)                  # deterministic
    assert torch.equal(c_pk, c_exact)
    ref = torch.zeros(Q, FS0, D, dtype=torch.float64)
    xc, dc = x.cpu(), da.double().cpu()
    for k in range(FS0):
        ref[:, k].index_add_(0, xc[:, k:k + Tl].reshape(-1), dc)
    # the kernel's scale, recomputed: every term is rounded to 1 / S, and an entry (q, k) sums
    # at most count(q) terms, so its error is within count_max / (2 S) of the exact sum (then
    # rounded to bf16)
    import math
    amax = float(da.float().abs().max())
    cmax = int(torch.bincount(xc.reshape(-1), minlength=Q).max())
    S = 2.0 ** min(math.floor(math.log2(2.0 ** 30 / (amax * cmax))), 40)
    err = (t_pk.double() - ref).abs()
    bound = ref.abs() * 2.0 ** -8 + cmax / (2 * S) + 1e-12
    worst = float((err / bound).max())
    diff = (t_pk - t_exact).abs()
    frac = float((diff > 0).double().mean())
    print('S = 2^%d, count max %d: packed vs exact %.5f of entries apart; worst error %.3f of '
          'the bound' % (math.log2(S), cmax, frac, worst))
    assert worst <= 1.0
    # on average the packed result is as close to the fp64 sums as the exact path's bf16 output
    # (measured: 0.6 % of the entries one bf16 step from the exact path's on uniform indices,
    #  7-17 % under the 60 % skew, whose scale is 8-16x coarser: a tenth of a bf16 step of
    #  pre-rounding error flips that many roundings)
    e_pk = float(err.mean())
    e_ex = float((t_exact.double() - ref).abs().mean())
    print('mean abs error vs fp64: packed %.3e, exact path %.3e' % (e_pk, e_ex))
    assert e_pk <= 1.5 * e_ex + 1e-12


def _dtab4(hip, da, x, B, Tl, blk=None, amax=None, want_colsum=True):
    import ctypes
    FS0, Q, D = 16, 256, da.shape[1]
    work = torch.empty(Q * FS0 * D, device=DEV, dtype=torch.int64)
    tab = torch.empty(Q, FS0, D, device=DEV, dtype=torch.bfloat16)
    colsum = torch.full((FS0 * D,), 7.0, device=DEV)
    done = ctypes.c_int(-1)
    hip.lib().call('srnn_mlp_dtab4', hip.BF16, hip.ptr(da), D, hip.ptr(x), x.shape[1], 0, B, Tl,
                   hip.ptr(tab), hip.BF16, D, FS0, Q, hip.ptr(work), work.numel() * 8,
                   hip.ptr(colsum), ctypes.byref(done), hip.ptr(amax), hip.ptr(blk), hip.stream())
    torch.cuda.synchronize()
    if want_colsum:
        assert done.value == 1
        return tab.cpu(), colsum.cpu()
    return tab.cpu(), (colsum.cpu() if done.value == 1 else None)


@pytest.mark.parametrize('B,Tl', [(64, 1024), (3, 37)])
def test_mlp_dtab_blocked_operand_bit_identical(hip, B, Tl):
    """srnn_mlp_dtab4 reading the column-blocked copy blk[D/4][B*Tl][4] gives the same dTab and
    column sums as reading the row-major da, bit for bit."""
    D = 1024
    g = torch.Generator().manual_seed(B + Tl)
    x = torch.randint(0, 256, (B, Tl + 15), generator=g).to(DEV)
    da = (torch.randn(B * Tl, D, generator=g) * 1e-3).to(DEV, torch.bfloat16)
    blk = da.reshape(B * Tl, D // 4, 4).permute(1, 0, 2).contiguous()
    t0, c0 = _dtab4(hip, da, x, B, Tl)
    t1, c1 = _dtab4(hip, da, x, B, Tl, blk=blk)
    assert torch.equal(t0, t1) and torch.equal(c0, c1)


def test_gemm_writes_blocked_copy(hip):
    """srnn_gemm_amax_blk_next: the ReLU-masked bf16 GEMM producing da1 also writes its output
    column-blocked ([N/4][M][4]) and max |C|; the copy is the output, permuted, bit for bit
    (the da1 GEMM's shape class: M = B T rows, a 256-tile grid that fills the chip)."""
    M, N, K = 65536, 1024, 512
    g = torch.Generator().manual_seed(5)
    A = (torch.randn(M, K, generator=g)).to(DEV, torch.bfloat16)
    W = (torch.randn(N, K, generator=g) * 0.05).to(DEV, torch.bfloat16)
    mask = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    amax = torch.zeros(1, device=DEV, dtype=torch.int32)
    blk = torch.full((N // 4, M, 4), float('nan'), device=DEV, dtype=torch.bfloat16)
    hip.lib().call('srnn_gemm_amax_blk_next', hip.ptr(amax), hip.ptr(blk))
    C = hip.gemm(A, W, transB=True, mask=mask, out_dtype=torch.bfloat16)
    taken = hip.lib().dll.srnn_gemm_amax_taken()
    torch.cuda.synchronize()
    assert taken == 2
    ref = C.reshape(M, N // 4, 4).permute(1, 0, 2)
    assert torch.equal(blk.view(torch.int16), ref.contiguous().view(torch.int16))
    assert amax.view(torch.float32).item() == C.float().abs().max().item()


@pytest.mark.parametrize('B,Tl', [(128, 1024), (64, 2048), (16, 9000)])
def test_mlp_dtab_skew_takes_exact_form(hip, B, Tl):
    """A sample histogram past the packed form's precision bound (one value at > 65,536
    positions: long silences at large B) makes the gated exact 2^-40 form produce dTab:
    bit-identical to SRNN_DTAB_PACK=0's output.  Tl = 9000 is past the exact position-major
    form's LDS budget (the packed one still fits): the packed form must not be taken there,
    since nothing would stand behind it."""
    import os
    D = 1024
    g = torch.Generator().manual_seed(11 + Tl)
    x = torch.randint(0, 256, (B, Tl + 15), generator=g)
    x[torch.rand(x.shape, generator=g) < 0.6] = 128
    assert int(torch.bincount(x.reshape(-1)).max()) > 65536
    x = x.to(DEV)
    da = (torch.randn(B * Tl, D, generator=g) * 1e-4).to(DEV, torch.bfloat16)
    t_gate, c_gate = _dtab4(hip, da, x, B, Tl, want_colsum=False)
    os.environ['SRNN_DTAB_PACK'] = '0'
    try:
        t_ex, c_ex = _dtab4(hip, da, x, B, Tl, want_colsum=False)
    finally:
        del os.environ['SRNN_DTAB_PACK']
    assert torch.equal(t_gate.view(torch.int16), t_ex.view(torch.int16))
    assert (c_gate is None) == (c_ex is None)
    if c_gate is not None:
        assert torch.equal(c_gate, c_ex)
    if Tl > 8000:
        # every entry is a real sum (no stale workspace): compare with an fp64 scatter
        ref = torch.zeros(256, 16, D, dtype=torch.float64)
        xc, dc = x.cpu(), da.double().cpu()
        for k in range(16):
            ref[:, k].index_add_(0, xc[:, k:k + Tl].reshape(-1), dc)
        err = (t_gate.double() - ref).abs()
        assert float((err - ref.abs() * 2.0 ** -8).max()) < 1e-6


def test_mlp_dtab_nonfinite_poisons(hip):
    """A NaN in da (packed form): dTab and the column sums come out NaN, not integers."""
    B, Tl, D = 4, 256, 1024
    g = torch.Generator().manual_seed(12)
    x = torch.randint(0, 256, (B, Tl + 15), generator=g).to(DEV)
    da = (torch.randn(B * Tl, D, generator=g) * 1e-3).to(DEV, torch.bfloat16)
    da[5, 17] = float('nan')
    t, c = _dtab4(hip, da, x, B, Tl)
    assert torch.isnan(t.float()).all() and torch.isnan(c).all()


def test_dtab_blocked_step_bit_identical(hip, monkeypatch):
    """A bf16 TBPTT step at D = 1024 with the da1 GEMM's blocked copy feeding the scatter
    (default) equals the row-major-operand step (SRNN_DTAB_BLK=0) bit for bit."""
    import model as M
    import nn as snn
    outs = []
    for flag in ('0', '1'):
        monkeypatch.setenv('SRNN_DTAB_BLK', flag)
        torch.manual_seed(3)
        m = M.SampleRNN([16, 4], 1, 1024, True, 256, True, False, 43, 6)
        m.compute_dtype = torch.bfloat16
        pred = M.Predictor(m).to(DEV)
        B, T, L = 4, 1024, 64
        g = torch.Generator().manual_seed(4)
        inp = torch.randint(0, 256, (B, L + T - 1), generator=g).to(DEV)
        tgt = torch.randint(0, 256, (B, T), generator=g).to(DEV)
        cond = torch.rand(B, T // L, 43, generator=g).to(DEV)
        spk = torch.arange(B).reshape(-1, 1).to(DEV) % 6
        loss = snn.sequence_nll_loss_bits(pred(inp, True, cond, spk), tgt)
        loss.backward()
        outs.append({k: p.grad.detach().cpu().clone() for k, p in pred.named_parameters()
                     if p.grad is not None})
    assert outs[0].keys() == outs[1].keys()
    for k in outs[0]:
        assert torch.equal(outs[0][k], outs[1][k]), k


def test_fused_upsampling_bias_grad_in_step(hip):
    """A bf16 TBPTT step at D = 1024 takes the bottom tier's upsampling bias gradient from the
    MLP's dTab pass (no separate column sum), and it equals the column sum of d(upper)."""
    import model as M
    import nn as snn
    torch.manual_seed(3)
    m = M.SampleRNN([16, 4], 1, 1024, True, 256, True, False, 43, 6)
    m.compute_dtype = torch.bfloat16
    pred = M.Predictor(m).to(DEV)
    B, T, L = 2, 128, 64
    g = torch.Generator().manual_seed(4)
    inp = torch.randint(0, 256, (B, L + T - 1), generator=g).to(DEV)
    tgt = torch.randint(0, 256, (B, T), generator=g).to(DEV)
    cond = torch.rand(B, T // L, 43, generator=g).to(DEV)
    spk = torch.tensor([[1], [4]], device=DEV)
    before = M._STATS['fused_colsum']
    lp = pred(inp, True, cond, spk)
    snn.sequence_nll_loss_bits(lp, tgt).backward()
    assert M._STATS['fused_colsum'] == before + 1
    bot = m.frame_level_rnns[0]
    grad_fused = bot.upsampling.bias.grad.clone()
    # same step with the column sum computed by the tier (attribute stripped by a clone)
    for p in pred.parameters():
        p.grad = None
    pred.reset_hidden_states()
    lp = pred(inp, True, cond, spk)
    loss = snn.sequence_nll_loss_bits(lp, tgt)
    orig = M.mlp_backward

    def strip(ctx, dlogp, nll=None):
        d_upper, grads = orig(ctx, dlogp, nll)
        return d_upper.clone(), grads
    M.mlp_backward = strip
    try:
        loss.backward()
    finally:
        M.mlp_backward = orig
    torch.testing.assert_close(bot.upsampling.bias.grad, grad_fused, atol=1e-7, rtol=1e-5)


def test_upper_tier_reuses_lower_bf16_gradient(hip):
    """bf16 step: the top tier's upsampling backward takes the compute-dtype copy of its
    output gradient from the bottom tier (which cast its dx0 for its own weight gradients)
    instead of casting again; every top-tier gradient equals the un-fused step's bit for bit."""
    import model as M
    import nn as snn
    torch.manual_seed(5)
    m = M.SampleRNN([16, 4], 1, 1024, True, 256, True, False, 43, 6)
    m.compute_dtype = torch.bfloat16
    pred = M.Predictor(m).to(DEV)
    B, T, L = 2, 128, 64
    g = torch.Generator().manual_seed(6)
    inp = torch.randint(0, 256, (B, L + T - 1), generator=g).to(DEV)
    tgt = torch.randint(0, 256, (B, T), generator=g).to(DEV)
    cond = torch.rand(B, T // L, 43, generator=g).to(DEV)
    spk = torch.tensor([[2], [5]], device=DEV)
    top = m.frame_level_rnns[1]
    grads = []
    for fused in (True, False):
        for p in pred.parameters():
            p.grad = None
        pred.reset_hidden_states()
        before = M._STATS['fused_lp']
        loss = snn.sequence_nll_loss_bits(pred(inp, True, cond, spk), tgt)
        orig = M.tier_backward

        def strip(ctx, dY, need_h0):
            if hasattr(dY, '_srnn_lp'):
                del dY._srnn_lp
            return orig(ctx, dY, need_h0)
        if not fused:
            M.tier_backward = strip
        try:
            loss.backward()
        finally:
            M.tier_backward = orig
        assert M._STATS['fused_lp'] == before + (1 if fused else 0)
        grads.append({k: p.grad.clone() for k, p in top.named_parameters() if p.grad is not None})
    assert grads[0].keys() == grads[1].keys()
    for k in grads[0]:
        assert torch.equal(grads[0][k], grads[1][k]), k


@pytest.mark.parametrize('perm',[(0, 1, 2), (0, 2, 1), (1, 0, 2), (1, 2, 0), (2, 0, 1),
                                  (2, 1, 0)])
@pytest.mark.parametrize('shape', [(3, 37, 70), (16, 64, 33), (1, 1, 5)])
def test_permute3(hip, perm, shape):
    x = _rand(*shape, seed=sum(shape)).to(DEV)
    ref = x.permute(perm).contiguous()
    torch.testing.assert_close(hip.permute3(x, perm), ref, atol=0, rtol=0)
    torch.testing.assert_close(hip.permute3(x, perm, dtype=torch.bfloat16), ref.to(torch.bfloat16),
                               atol=0, rtol=0)
    acc = _rand(*ref.shape, seed=3).to(DEV)
    want = acc + ref
    hip.permute3(x, perm, out=acc, accumulate=True)
    torch.testing.assert_close(acc, want, atol=0, rtol=0)


@pytest.mark.parametrize('B,Tl,D', [(128, 1024, 1024), (4, 2048, 1024), (6, 1000, 512),
                                    (3, 4096, 272)])
def test_mlp_l1_lds_matches_l2_gather(hip, B, Tl, D, monkeypatch):
    """bf16 training gather: the LDS-resident table kernel == the L2-gather kernels bit for
    bit (same summation order, single-rounding adds)."""
    FS0, Q = 16, 256
    g = torch.Generator().manual_seed(B + Tl + D)
    tab = (torch.randn(FS0, Q, D, generator=g) * 0.3).to(DEV, torch.bfloat16)
    x = torch.randint(0, Q, (B, Tl + FS0 + 3), generator=g).to(DEV)
    upper = (torch.randn(B * Tl, D, generator=g) * 0.5).to(DEV, torch.bfloat16)
    outs = []
    for flag in ('1', '0'):
        monkeypatch.setenv('SRNN_L1_LDS', flag)
        out = torch.empty(B * Tl, D, device=DEV, dtype=torch.bfloat16)
        hip.lib().call('srnn_mlp_l1', hip.BF16, hip.ptr(tab), hip.ptr(x), x.shape[1], 2, B, Tl,
                       hip.BF16, hip.ptr(upper), D, hip.ptr(out), D, D, FS0, Q, hip.stream())
        outs.append(out)
    torch.testing.assert_close(outs[0], outs[1], atol=0, rtol=0)
    idx = torch.stack([x[:, 2 + k:2 + k + Tl] for k in range(FS0)], -1).reshape(B * Tl, FS0)
    ref = upper.float().clone()
    for k in range(FS0):
        ref += tab[k].float()[idx[:, k]]
    torch.testing.assert_close(outs[0].float(), ref.clamp_min(0).to(torch.bfloat16).float(),
                               atol=2e-2, rtol=1e-2)


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('rows,cols', [(131072, 256), (8192, 1024), (100, 37), (1, 1030), (0, 8),
                                       (5000, 16384), (131072, 1), (5000, 3), (7, 2)])
def test_colsum(hip, dtype, rows, cols):
    x = _rand(max(rows, 1), cols + 4, seed=rows + cols)[:rows].to(DEV, dtype)
    view = x[:, 2:cols + 2] if dtype == torch.float32 else x[:, :cols]
    ref = view.double().sum(0).float().cpu()
    out = hip.colsum(view, rows, cols, lds=x.stride(0))
    torch.testing.assert_close(out.cpu(), ref, atol=1e-5 * max(rows, 1) ** 0.5, rtol=1e-5)
    out2 = torch.ones(cols, device=DEV)
    hip.colsum(view, rows, cols, lds=x.stride(0), out=out2, alpha=0.5, accumulate=True)
    torch.testing.assert_close(out2.cpu(), 1 + 0.5 * ref, atol=1e-5 * max(rows, 1) ** 0.5,
                               rtol=1e-5)


def test_adam_clip_multi_matches_torch(hip):
    """Multi-tensor launch: 70 tensors (two launches of <= 64) of ragged sizes, 3 steps."""
    import ctypes
    sizes = [1, 3, 7, 64, 1000, 2049, 4096, 10007] * 9
    sizes = sizes[:70]
    ps = [_rand(n, seed=i).to(DEV) for i, n in enumerate(sizes)]
    ms = [torch.zeros(n, device=DEV) for n in sizes]
    vs = [torch.zeros(n, device=DEV) for n in sizes]
    refs = [p.detach().cpu().clone().requires_grad_(True) for p in ps]
    opt = torch.optim.Adam(refs, lr=1e-3)
    arr = lambda ts: (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])  # noqa: E731
    for step in range(1, 4):
        gs = [_rand(n, scale=3.0, seed=100 * step + i) for i, n in enumerate(sizes)]
        gd = [g.to(DEV) for g in gs]
        hip.lib().call('srnn_adam_clip_multi', len(sizes), arr(ps), arr(gd), arr(ms), arr(vs), None,
                       (ctypes.c_int64 * len(sizes))(*sizes), -1.0, 1.0, 1e-3, 0.9, 0.999, 1e-8,
                       step, hip.stream())
        for r, g in zip(refs, gs):
            r.grad = g.clamp(-1, 1)
        opt.step()
        for g, d in zip(gs, gd):
            torch.testing.assert_close(d.cpu(), g.clamp(-1, 1))
    for p, r in zip(ps, refs):
        torch.testing.assert_close(p.cpu(), r.detach(), atol=1e-7, rtol=1e-6)


def test_adam_clip_multi_empty_tensors_across_chunks(hip):
    """> 64 tensors with empty ones among them: each chunk of 64 non-empty tensors starts
    where the previous chunk's scan stopped, so no tensor is updated twice or skipped."""
    import ctypes
    sizes = []
    for i in range(150):
        sizes.append(0 if i % 7 == 3 else 1 + (i * 37) % 3000)
    ps = [_rand(max(n, 1), seed=i)[:n].contiguous().to(DEV) for i, n in enumerate(sizes)]
    ms = [torch.zeros(n, device=DEV) for n in sizes]
    vs = [torch.zeros(n, device=DEV) for n in sizes]
    refs = [p.detach().cpu().clone().requires_grad_(True) for p in ps]
    opt = torch.optim.Adam([r for r in refs if r.numel()], lr=1e-3)
    gs = [_rand(max(n, 1), scale=3.0, seed=500 + i)[:n].contiguous() for i, n in enumerate(sizes)]
    gd = [g.to(DEV) for g in gs]
    arr = lambda ts: (ctypes.c_void_p * len(ts))(*[t.data_ptr() if t.numel() else None  # noqa
                                                   for t in ts])
    hip.lib().call('srnn_adam_clip_multi', len(sizes), arr(ps), arr(gd), arr(ms), arr(vs), None,
                   (ctypes.c_int64 * len(sizes))(*sizes), -1.0, 1.0, 1e-3, 0.9, 0.999, 1e-8, 1,
                   hip.stream())
    for r, g in zip(refs, gs):
        r.grad = g.clamp(-1, 1)
    opt.step()
    for p, r in zip(ps, refs):
        torch.testing.assert_close(p.cpu(), r.detach(), atol=1e-7, rtol=1e-6)


def test_adam_clip_matches_torch(hip):
    n = 10007
    p0 = _rand(n, seed=1)
    p = p0.clone().to(DEV)
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    pr = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([pr], lr=1e-3)
    for step in range(1, 4):
        g = _rand(n, scale=3.0, seed=10 + step)
        gd = g.to(DEV)
        hip.lib().call('srnn_adam_clip', hip.ptr(p), hip.ptr(gd), hip.ptr(m), hip.ptr(v), None, n,
                       -1.0, 1.0, 1e-3, 0.9, 0.999, 1e-8, step, hip.stream())
        pr.grad = g.clamp(-1, 1)
        opt.step()
        torch.testing.assert_close(gd.cpu(), g.clamp(-1, 1))
    torch.testing.assert_close(p.cpu(), pr.detach(), atol=1e-7, rtol=1e-6)


def test_weight_norm(hip):
    g = (torch.rand(20, 1, 1) + 0.5).to(DEV)
    v = _rand(20, 7, 3, seed=3).to(DEV)
    w = hip.weight_norm(g, v)
    ref = v.cpu() * (g.cpu().reshape(-1) / v.cpu().reshape(20, -1).norm(dim=1)).reshape(-1, 1, 1)
    torch.testing.assert_close(w.cpu(), ref, atol=1e-6, rtol=1e-6)
    gg = g.cpu().clone().requires_grad_(True)
    vv = v.cpu().clone().requires_grad_(True)
    ww = vv * (gg.reshape(-1) / vv.reshape(20, -1).norm(dim=1)).reshape(-1, 1, 1)
    dw = _rand(20, 7, 3, seed=4)
    ww.backward(dw)
    dg, dv = hip.weight_norm_bwd(g, v, dw.to(DEV))
    torch.testing.assert_close(dg.cpu(), gg.grad, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(dv.cpu(), vv.grad, atol=1e-5, rtol=1e-5)


def test_learned_upsampling_module(hip):
    import nn as snn
    torch.manual_seed(0)
    m = snn.LearnedUpsampling1d(24, 16, 4).to(DEV)
    with torch.no_grad():
        m.bias.uniform_(-0.1, 0.1)
    x = _rand(3, 24, 5, seed=2).to(DEV).requires_grad_(True)
    y = m(x)
    xr = x.detach().cpu().requires_grad_(True)
    Wr = m.conv_t.weight.detach().cpu().requires_grad_(True)
    br = m.bias.detach().cpu().requires_grad_(True)
    ref = torch.nn.functional.conv_transpose1d(xr, Wr, stride=4) + \
        br.unsqueeze(0).unsqueeze(2).expand(3, 16, 5, 4).reshape(3, 16, 20)
    torch.testing.assert_close(y.detach().cpu(), ref.detach(), atol=1e-5, rtol=1e-5)
    dy = _rand(3, 16, 20, seed=5)
    y.backward(dy.to(DEV))
    ref.backward(dy)
    torch.testing.assert_close(x.grad.cpu(), xr.grad, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(m.conv_t.weight.grad.cpu(), Wr.grad, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(m.bias.grad.cpu(), br.grad, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize('Cin,Cout,k', [(1024, 1024, 16), (128, 64, 4), (64, 96, 2)])
def test_convt_fold_matches_weight_norm_permute(hip, Cin, Cout, k):
    """W_up = (g v / ||v||).permute(2, 1, 0) straight from v: bit-identical to the weight-norm
    kernel followed by the permute (same per-channel scale), fp32 and bf16."""
    g = (torch.rand(Cin, 1, 1) + 0.5).to(DEV)
    v = _rand(Cin, Cout, k, seed=Cin + k).to(DEV)
    ref = hip.permute3(hip.weight_norm(g, v), (2, 1, 0))
    for dt in (torch.float32, torch.bfloat16):
        out = hip.convt_operand(g, v, k, dt)
        torch.testing.assert_close(out, ref.to(dt), atol=0, rtol=0)
    plain = hip.convt_operand(None, v, k, torch.float32)
    torch.testing.assert_close(plain, hip.permute3(v, (2, 1, 0)), atol=0, rtol=0)


@pytest.mark.parametrize('Cin,Cout,k', [(1024, 1024, 16), (256, 1024, 4), (20, 12, 3)])
def test_convt_wn_bwd_matches_weight_norm_bwd(hip, Cin, Cout, k):
    """Per-channel weight-norm backward from the transposed GEMM gradient [i][j*Cout + o]
    == weight_norm_bwd on the permuted gradient, bit for bit."""
    g = (torch.rand(Cin, 1, 1) + 0.5).to(DEV)
    v = _rand(Cin, Cout, k, seed=11).to(DEV)
    dwt = _rand(Cin, k * Cout, seed=12).to(DEV)
    dw = hip.permute3(dwt.reshape(Cin, k, Cout), (0, 2, 1))
    dg_ref, dv_ref = hip.weight_norm_bwd(g, v, dw)
    dg, dv = hip.convt_wn_bwd(g, v, dwt, k)
    torch.testing.assert_close(dg, dg_ref, atol=0, rtol=0)
    torch.testing.assert_close(dv, dv_ref, atol=0, rtol=0)


@pytest.mark.parametrize('B,T', [(4, 1024), (3, 17)])
def test_nll_bwd_dense_gradient(hip, B, T):
    """srnn_nll_bwd (vectorised Q = 256 path): -scale * g at the target, zero elsewhere."""
    Q = 256
    tgt = torch.randint(0, Q, (B, T), generator=torch.Generator().manual_seed(B + T))
    gd = torch.full((1,), 0.75, device=DEV)
    d = torch.full((B, T, Q), float('nan'), device=DEV)
    tgd = tgt.to(DEV)
    hip.lib().call('srnn_nll_bwd', hip.ptr(tgd), T, T, B * T, Q, hip.ptr(d), Q, 0.5, hip.ptr(gd),
                   hip.stream())
    ref = torch.zeros(B, T, Q)
    ref.scatter_(2, tgt.unsqueeze(-1), -0.375)
    torch.testing.assert_close(d.cpu(), ref, atol=0, rtol=0)


@pytest.mark.parametrize('B,D,Fr', [(128, 1024, 64), (100, 256, 9)])
def test_gru_xcd_bwd2_lowp_outputs(hip, B, D, Fr):
    """srnn_gru_xcd_bwd2 without fp32 dgh/dgi: dgh_lp and dgi_lp equal the bf16 casts of the
    fp32 sweep's outputs, bsum the per-row sums over t of [dar | daz | dghn | dan]."""
    T = torch.bfloat16
    nb = hip.gru_xcd_bwd_work_bytes(T, B, D)
    if not nb:
        pytest.skip('gru_xcd not supported on this device')
    g = torch.Generator().manual_seed(B + D)
    whh = (torch.randn(3 * D, D, generator=g) * 0.03).to(T)
    bhh = torch.randn(3 * D, generator=g) * 0.1
    gi = torch.randn(B * Fr, 3 * D, generator=g) * 0.5
    h0 = torch.randn(B, D, generator=g) * 0.5
    dy = (torch.randn(B, Fr, D, generator=g) * 0.1).to(DEV)
    out, gates = _gru_ref(gi, h0, whh, bhh, Fr)
    whh_t = whh.float().t().contiguous().to(DEV, T)
    gtd, outd, h0d = gates.to(DEV), out.to(DEV), h0.to(DEV)

    def run(full):
        dgh = torch.full((B, Fr, 3 * D), float('nan'), device=DEV) if full else None
        dgi = torch.full((B, Fr, 3 * D), float('nan'), device=DEV) if full else None
        dgh_lp = torch.zeros((B, Fr, 3 * D), device=DEV, dtype=T)
        dgi_lp = None if full else torch.zeros((B, Fr, 3 * D), device=DEV, dtype=T)
        bsum = None if full else torch.full((B, 4 * D), float('nan'), device=DEV)
        ddir0 = torch.full((B, D), float('nan'), device=DEV)
        work = torch.full((nb,), 7, device=DEV, dtype=torch.uint8)
        hip.lib().call('srnn_gru_xcd_bwd2', hip.BF16, B, D, Fr, hip.ptr(dy), Fr * D, D,
                       hip.ptr(gtd), Fr * 4 * D, 4 * D, hip.ptr(outd), Fr * D, D, hip.ptr(h0d),
                       hip.ptr(whh_t), hip.ptr(dgh), hip.ptr(dgh_lp), hip.ptr(dgi),
                       hip.ptr(dgi_lp), hip.ptr(bsum), Fr * 3 * D, 3 * D, hip.ptr(ddir0),
                       hip.ptr(work), nb, hip.stream())
        torch.cuda.synchronize()
        assert hip.lib().dll.srnn_gru_xcd_error(hip.ptr(work)) == 0
        return dgh, dgi, dgh_lp, dgi_lp, bsum, ddir0

    dgh, dgi, dgh_lp_a, _, _, ddir_a = run(True)
    _, _, dgh_lp, dgi_lp, bsum, ddir_b = run(False)
    torch.testing.assert_close(dgh_lp, dgh_lp_a, atol=0, rtol=0)
    torch.testing.assert_close(dgi_lp, dgi.to(T), atol=0, rtol=0)
    torch.testing.assert_close(ddir_b, ddir_a, atol=0, rtol=0)
    ref = torch.cat([dgh.sum(1), dgi[..., 2 * D:].sum(1)], 1)
    torch.testing.assert_close(bsum, ref, atol=1e-5 * ref.abs().max().item(), rtol=1e-5)


def test_bf16_parameter_copies_follow_adam(hip):
    """The cached bf16 parameter copies (samplernn_hip.cast_param) stay equal to a fresh cast
    of the fp32 parameters across fused clip+Adam steps (the Adam kernel rewrites them), and
    a torch in-place edit of a parameter invalidates its copy."""
    import model as M
    import nn as snn
    import optim
    torch.manual_seed(5)
    m = M.SampleRNN([16, 4], 1, 256, True, 256, True, False, 43, 6)
    m.compute_dtype = torch.bfloat16
    pred = M.Predictor(m).to(DEV)
    opt = optim.gradient_clipping(torch.optim.Adam(pred.parameters(), lr=1e-3))
    B, T, L = 2, 128, 64
    g = torch.Generator().manual_seed(6)
    for step in range(3):
        inp = torch.randint(0, 256, (B, L + T - 1), generator=g).to(DEV)
        tgt = torch.randint(0, 256, (B, T), generator=g).to(DEV)
        cond = torch.rand(B, T // L, 43, generator=g).to(DEV)
        spk = torch.tensor([[1], [4]], device=DEV)
        opt.zero_grad()

        def closure():
            loss = snn.sequence_nll_loss_bits(pred(inp, step == 0, cond, spk), tgt)
            loss.backward()
            return loss
        opt.step(closure)
    torch.cuda.synchronize()
    n = 0
    for p in pred.parameters():
        c = hip.shadow_of(p)
        if c is not None:
            n += 1
            torch.testing.assert_close(c, p.detach().to(torch.bfloat16), atol=0, rtol=0)
    assert n >= 6
    w = m.sample_level_mlp.hidden.weight
    assert hip.shadow_of(w) is not None
    with torch.no_grad():
        w.mul_(0.5)
    assert hip.shadow_of(w) is None
    torch.testing.assert_close(hip.cast_param(w, torch.bfloat16), w.detach().to(torch.bfloat16),
                               atol=0, rtol=0)


def _bits_ref(a):
    """ReLU mask bits of a (M, N) in the srnn_gemm_bits layout, as int16 (M, N / 16)."""
    pos = (a.float() > 0).to(torch.int32).reshape(a.shape[0], -1, 16)
    w = (pos << torch.arange(16, device=a.device, dtype=torch.int32)).sum(-1)
    return w.to(torch.int32).view(-1).to(torch.int16).reshape(a.shape[0], -1)


@pytest.mark.parametrize('B,Tl,D', [(128, 1024, 1024), (3, 4096, 272), (6, 1000, 512)])
def test_mlp_l1_bits(hip, B, Tl, D, monkeypatch):
    """a1 with its ReLU mask as bits (the LDS kernel's fused bits, and the bits pass after the
    other gathers) == the plain gather's a1 and the bits of that a1."""
    FS0, Q = 16, 256
    g = torch.Generator().manual_seed(B * 7 + D)
    tab = (torch.randn(FS0, Q, D, generator=g) * 0.3).to(DEV, torch.bfloat16)
    x = torch.randint(0, Q, (B, Tl + FS0 + 3), generator=g).to(DEV)
    upper = (torch.randn(B * Tl, D, generator=g) * 0.5).to(DEV, torch.bfloat16)
    ref = torch.empty(B * Tl, D, device=DEV, dtype=torch.bfloat16)
    hip.lib().call('srnn_mlp_l1', hip.BF16, hip.ptr(tab), hip.ptr(x), x.shape[1], 2, B, Tl,
                   hip.BF16, hip.ptr(upper), D, hip.ptr(ref), D, D, FS0, Q, hip.stream())
    for flag in ('1', '0'):
        monkeypatch.setenv('SRNN_L1_LDS', flag)
        out = torch.empty_like(ref)
        bits = hip.relu_bits(B * Tl, D, DEV)
        hip.lib().call('srnn_mlp_l1_bits', hip.ptr(tab), hip.ptr(x), x.shape[1], 2, B, Tl,
                       hip.ptr(upper), D, hip.ptr(out), D, D, FS0, Q, hip.ptr(bits),
                       bits.stride(0), hip.stream())
        torch.testing.assert_close(out, ref, atol=0, rtol=0)
        assert torch.equal(bits, _bits_ref(ref))


def _bits_grouped_ref(a):
    """The same bits in the grouped layout (u16 [N / 16][M], flat)."""
    return _bits_ref(a).t().reshape(-1).contiguous()


@pytest.mark.parametrize('B,Tl,D', [(16, 1024, 1024), (3, 4096, 272 - 16), (6, 1000, 512)])
def test_mlp_l1_bits_grouped(hip, B, Tl, D, monkeypatch):
    """a1's mask bits in the grouped layout (ldb = 0; the L1 LDS kernel's fused bits and the
    bits pass after the other gathers) == the grouped bits of the plain gather's a1."""
    FS0, Q = 16, 256
    g = torch.Generator().manual_seed(B * 5 + D)
    tab = (torch.randn(FS0, Q, D, generator=g) * 0.3).to(DEV, torch.bfloat16)
    x = torch.randint(0, Q, (B, Tl + FS0 + 3), generator=g).to(DEV)
    upper = (torch.randn(B * Tl, D, generator=g) * 0.5).to(DEV, torch.bfloat16)
    ref = torch.empty(B * Tl, D, device=DEV, dtype=torch.bfloat16)
    hip.lib().call('srnn_mlp_l1', hip.BF16, hip.ptr(tab), hip.ptr(x), x.shape[1], 2, B, Tl,
                   hip.BF16, hip.ptr(upper), D, hip.ptr(ref), D, D, FS0, Q, hip.stream())
    for flag in ('1', '0'):
        monkeypatch.setenv('SRNN_L1_LDS', flag)
        out = torch.empty_like(ref)
        bits = hip.relu_bits_grouped(B * Tl, D, DEV)
        hip.lib().call('srnn_mlp_l1_bits', hip.ptr(tab), hip.ptr(x), x.shape[1], 2, B, Tl,
                       hip.ptr(upper), D, hip.ptr(out), D, D, FS0, Q, hip.ptr(bits), 0,
                       hip.stream())
        torch.testing.assert_close(out, ref, atol=0, rtol=0)
        assert torch.equal(bits, _bits_grouped_ref(ref))


@pytest.mark.parametrize('M,N,K,amax', [(32768, 1024, 1024, True), (32768, 1024, 1024, False),
                                        (8192, 512, 192, True), (1024, 256, 128, True),
                                        (200, 128, 96, False),
                                        # K = 64 (one k-chunk per tile) with 2 tiles per
                                        # workgroup: the expanded fallback
                                        (131072, 256, 64, True), (131072, 256, 64, False),
                                        (131072, 256, 128, True)])
def test_gemm_mask_bits_grouped(hip, M, N, K, amax):
    """The grouped mask bits (the da1 GEMM's operand: staged by LDS-DMA in the bf16 pair-mode
    kernel, expanded to a mask on the other paths) == the bf16 mask tensor, bit for bit, with
    and without the max |C| request (the same maximum, taken by the same shapes)."""
    bf = torch.bfloat16
    A = _rand(M, K, seed=11).to(DEV, bf)
    W = _rand(N, K, seed=12).to(DEV, bf)                  # W^T stored k-contiguous (NT)
    act = _rand(M, N, seed=13).to(DEV, bf)
    act[act.float().abs() < 0.3] = 0.0
    bits = hip.relu_bits_grouped(M, N, DEV)
    hip.lib().call('srnn_relu_bits', hip.BF16, hip.ptr(act), N, M, N, hip.ptr(bits), 0,
                   hip.stream())
    assert torch.equal(bits, _bits_grouped_ref(act))
    res = []
    for kw in (dict(mask=act), dict(mask_bits=bits)):
        mx = torch.zeros(1, device=DEV, dtype=torch.int32)
        if amax:
            hip.lib().call('srnn_gemm_amax_next', hip.ptr(mx))
        o = hip.gemm(A, W, transB=True, out_dtype=bf, **kw)
        taken = hip.lib().dll.srnn_gemm_amax_taken() if amax else 0
        torch.cuda.synchronize()
        res.append((o, int(mx.item()), taken))
    assert torch.equal(res[0][0], res[1][0])
    assert res[0][2] == res[1][2]
    if res[0][2]:
        assert res[0][1] == res[1][1]
        ref = res[0][0].float().abs().max().item()
        assert res[1][1] == int(np.float32(ref).view(np.int32))
    if M * N >= 32768 * 1024 and K >= 128:
        assert res[1][2] == 1 or not amax                   # the LDS-staged kernel took it
    o3 = hip.gemm(A, W, transB=True, mask_bits=bits)       # fp32 out: the expanded fallback
    o4 = hip.gemm(A, W, transB=True, mask=act)
    assert torch.equal(o3, o4)


@pytest.mark.parametrize('M,N,K,tB,tile', [(1024, 512, 256, False, 5), (512, 1024, 1024, True, 5),
                                           (768, 512, 512, False, 5), (200, 144, 96, False, -1),
                                           (256, 256, 64, True, -1)])
def test_gemm_mask_bits(hip, M, N, K, tB, tile):
    """ReLU masks as bits: the masked GEMM with bits == with the bf16 mask tensor, bit for
    bit (256-tile kernel's bit epilogue, and the expanded-mask fallback of other shapes); the
    ReLU forward's bits_out == the bits of its bf16 output."""
    bf = torch.bfloat16
    A = _rand(M, K, seed=1).to(DEV, bf)
    W = (_rand(N, K, seed=2) if tB else _rand(K, N, seed=2)).to(DEV, bf)
    act = _rand(M, N, seed=3).to(DEV, bf)               # the layer's forward activation
    act[act.float().abs() < 0.3] = 0.0
    bits = hip.relu_bits(M, N, DEV)
    hip.lib().call('srnn_relu_bits', hip.BF16, hip.ptr(act), N, M, N, hip.ptr(bits),
                   bits.stride(0), hip.stream())
    assert torch.equal(bits, _bits_ref(act))
    o1 = hip.gemm(A, W, transB=tB, mask=act, out_dtype=bf, tile=tile)
    o2 = hip.gemm(A, W, transB=tB, mask_bits=bits, out_dtype=bf, tile=tile)
    assert torch.equal(o1, o2)
    o3 = hip.gemm(A, W, transB=tB, mask_bits=bits, tile=tile)     # fp32 out: fallback path
    o4 = hip.gemm(A, W, transB=tB, mask=act, tile=tile)
    assert torch.equal(o3, o4)
    bias = _rand(N, seed=4).to(DEV)
    bo = hip.relu_bits(M, N, DEV)
    y = hip.gemm(A, W, transB=tB, bias=bias, relu=True, out_dtype=bf, tile=tile, bits_out=bo)
    y0 = hip.gemm(A, W, transB=tB, bias=bias, relu=True, out_dtype=bf, tile=tile)
    assert torch.equal(y, y0)
    assert torch.equal(bo, _bits_ref(y))


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_fused_nll_logsoftmax_backward_bit_identical(hip, monkeypatch, dtype):
    """sequence_nll_loss_bits on the MLP's log-probs hands the MLP its gradient in closed form
    (srnn_nll_logsoftmax_bwd: dz = c (exp(logp) - onehot)); every gradient equals the
    two-kernel path's (dense fp32 dlogp + log-softmax backward) bit for bit.  Using the
    log-probs twice (another gradient summed onto the placeholder) raises instead of
    returning a wrong gradient."""
    import model as M
    import nn as snn
    torch.manual_seed(4)
    m = M.SampleRNN([16, 4], 1, 256, True, 256, True, False, 43, 6)
    m.compute_dtype = dtype
    pred = M.Predictor(m).to(DEV)
    B, T, L = 3, 256, 64
    g = torch.Generator().manual_seed(5)
    x = torch.randint(0, 256, (B, L + T), generator=g).to(DEV)
    cond = torch.rand(B, T // L, 43, generator=g).to(DEV)
    spk = (torch.arange(B) % 6).reshape(-1, 1).to(DEV)
    res = []
    for fused in (True, False):
        monkeypatch.setattr(snn, 'FUSED_NLL', fused)
        for p in pred.parameters():
            p.grad = None
        loss = snn.sequence_nll_loss_bits(pred(x[:, :-1], True, cond, spk), x[:, L:])
        loss.backward()
        res.append((float(loss), {k: p.grad.clone() for k, p in pred.named_parameters()
                                  if p.grad is not None}))
    assert res[0][0] == res[1][0]
    assert res[0][1].keys() == res[1][1].keys()
    for k in res[0][1]:
        assert torch.equal(res[0][1][k], res[1][1][k]), k
    monkeypatch.setattr(snn, 'FUSED_NLL', True)
    lp = pred(x[:, :-1], True, cond, spk)
    loss = snn.sequence_nll_loss_bits(lp, x[:, L:]) + lp.sum() * 0.0
    with pytest.raises(RuntimeError, match='used twice'):
        loss.backward()


def test_gemm_amax_request(hip):
    """srnn_gemm_amax_next: the next bf16-output GEMM on the gemm3 path also writes max |C|
    (as float bits) -- exactly the max of the bf16 values it stored; a GEMM that takes another
    path leaves the request untaken."""
    g = torch.Generator().manual_seed(11)
    a = (torch.randn(8192, 1024, generator=g)).to(DEV, torch.bfloat16)
    w = (torch.randn(1024, 1024, generator=g) * 0.05).to(DEV, torch.bfloat16)
    mask = (torch.rand(8192, 1024, generator=g) > 0.5).to(DEV, torch.bfloat16)
    amax = torch.zeros(1, device=DEV, dtype=torch.int32)
    hip.lib().call('srnn_gemm_amax_next', hip.ptr(amax))
    c = hip.gemm(a, w, mask=mask, out_dtype=torch.bfloat16)
    assert hip.lib().dll.srnn_gemm_amax_taken() == 1
    torch.cuda.synchronize()
    got = amax.view(torch.float32).item()
    assert got == c.float().abs().max().item()
    # a small GEMM (not on the 256 x 256 path) does not take the request
    amax.zero_()
    hip.lib().call('srnn_gemm_amax_next', hip.ptr(amax))
    hip.gemm(a[:64, :64].contiguous(), w[:64, :64].contiguous(), out_dtype=torch.bfloat16)
    assert hip.lib().dll.srnn_gemm_amax_taken() == 0


@pytest.mark.parametrize('form', ['nt_mask', 'nn_plain', 'nt_bias_relu'])
def test_gemm_csum_request(hip, form):
    """srnn_gemm_csum_next: the next bf16-output GEMM on the gemm3 pair path also writes the
    column sums of the bf16 values it stored, per 128-row block (part[M / 128][N]): each block
    row equals the fp64 sum of those stored values within fp32 rounding (128 terms), and the
    product itself is bit-identical to the same GEMM without the request.  nt_mask is the
    MLP's da2 = (dz W_out^T) * relu' form (model.py:320); nn_plain a shape that otherwise takes
    the ring ping-pong (the request keeps it on the pair kernel).  A bit-mask GEMM and a
    small GEMM leave the request untaken."""
    g = torch.Generator().manual_seed(12)
    M, N, K = (8192, 1024, 256) if form != 'nn_plain' else (8192, 4096, 512)
    a = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    kw = dict(out_dtype=torch.bfloat16)
    if form == 'nn_plain':
        w = (torch.randn(K, N, generator=g) * 0.05).to(DEV, torch.bfloat16)
    else:
        w = (torch.randn(N, K, generator=g) * 0.05).to(DEV, torch.bfloat16)
        kw['transB'] = True
    if form == 'nt_mask':
        kw['mask'] = (torch.rand(M, N, generator=g) > 0.5).to(DEV, torch.bfloat16)
    elif form == 'nt_bias_relu':
        kw.update(bias=torch.randn(N, generator=g).to(DEV), relu=True)
    plain = hip.gemm(a, w, **kw)
    part = torch.full((M // 128, N), float('nan'), device=DEV)
    hip.lib().call('srnn_gemm_csum_next', hip.ptr(part))
    c = hip.gemm(a, w, **kw)
    assert hip.lib().dll.srnn_gemm_csum_taken() == 1
    torch.cuda.synchronize()
    assert torch.equal(c, plain)
    ref = c.double().reshape(M // 128, 128, N).sum(1)
    mag = c.double().abs().reshape(M // 128, 128, N).sum(1)
    err = (part.double() - ref).abs()
    assert torch.isfinite(part).all()
    assert (err <= 128 * 2.0 ** -24 * mag + 1e-30).all(), float((err / (mag + 1e-30)).max())
    # bit masks (their own kernels) and a small GEMM do not take the request
    bits = torch.zeros((M, N // 16), device=DEV, dtype=torch.int16)
    hip.lib().call('srnn_gemm_csum_next', hip.ptr(part))
    hip.gemm(a, w, mask_bits=bits, **{k: v for k, v in kw.items() if k != 'mask'})
    assert hip.lib().dll.srnn_gemm_csum_taken() == 0
    hip.lib().call('srnn_gemm_csum_next', hip.ptr(part))
    hip.gemm(a[:64, :64].contiguous(), a[:64, :64].contiguous(), out_dtype=torch.bfloat16)
    assert hip.lib().dll.srnn_gemm_csum_taken() == 0


@pytest.mark.parametrize('S,n', [(6, 512), (5, 5000)])
def test_index_add_rows_deterministic(hip, S, n):
    """srnn_index_add_rows (the speaker-embedding gradient): table[q] += the rows of src whose
    index is q, summed in row order -- the same bits on every run, equal to a sequential fp32
    sum in that order, within fp32 rounding of the fp64 index_add (5000 rows: several LDS
    chunks; -0.0 in the table and in src keeps its sequential-order bits).  The device copies
    are held in names until the kernel has run: a temporary freed at the call could hand its
    block to the next one before the kernel reads it."""
    g = torch.Generator().manual_seed(21)
    idx = torch.randint(0, S, (n,), generator=g)
    src = torch.randn(n, S, generator=g)
    base = torch.randn(S, S, generator=g)
    base[0, :2] = -0.0
    src[::7, 1] = -0.0
    idx_d, src_d = idx.to(DEV), src.to(DEV)
    outs = []
    for _ in range(2):
        t = base.clone().to(DEV)
        hip.lib().call('srnn_index_add_rows', hip.ptr(t), S, S, hip.ptr(idx_d), n, S,
                       hip.ptr(src_d), S, hip.stream())
        torch.cuda.synchronize()
        outs.append(t.cpu())
    assert torch.equal(outs[0], outs[1])
    seq = base.clone()
    for r in range(n):                     # the kernel's order, in fp32
        seq[idx[r]] += src[r]
    assert torch.equal(outs[0], seq)
    ref = base.double().index_add(0, idx, src.double())
    torch.testing.assert_close(outs[0].double(), ref, atol=1e-5 if n <= 512 else 1e-4, rtol=0)


@pytest.mark.parametrize('args,kwargs', [((), {}), ((), {'reduction': 'sum'}),
                                         ((None, None, 7), {}), ((), {'reduction': 'none'}),
                                         ((), {'weight': 'w'}), ((), {'size_average': False}),
                                         ((), {'ignore_index': 300})])
def test_nll_bits_passes_nll_loss_arguments(hip, args, kwargs):
    """sequence_nll_loss_bits(input, target, *args, **kwargs) = nll_loss(input.view(-1, Q),
    target.view(-1), *args, **kwargs) * log2(e), as the reference (nn.py:66-70) -- the extra
    arguments are passed through instead of refused."""
    import math
    import nn as snn
    B, T, Q = 3, 40, 256
    g = torch.Generator().manual_seed(5)
    lp = torch.log_softmax(torch.randn(B, T, Q, generator=g), -1)
    tgt = torch.randint(0, Q, (B, T), generator=g)
    tgt[0, :5] = 7
    if kwargs.get('weight') == 'w':
        kwargs = {'weight': torch.rand(Q, generator=g)}
    ref = torch.nn.functional.nll_loss(lp.view(-1, Q), tgt.view(-1), *args, **kwargs) * \
        math.log(math.e, 2)
    dkw = {k: (v.to(DEV) if torch.is_tensor(v) else v) for k, v in kwargs.items()}
    got = snn.sequence_nll_loss_bits(lp.to(DEV), tgt.to(DEV), *args, **dkw)
    torch.testing.assert_close(got.cpu().double(), ref.double(), atol=2e-5, rtol=1e-5)


@pytest.mark.parametrize('out_dtype', [torch.bfloat16, torch.float32])
def test_gemm_batched_shared_operand_blaslt(hip, out_dtype):
    """Strided-batch GEMM with one operand shared by every batch (stride 0) -- the folded
    embedding . conv table build, Tab[k] = E . Wp[k]^T (model._build_tab) -- goes to hipBLASLt
    (round 6) and equals the per-batch fp32 products of the same bf16 operands."""
    Q, D, FS = 256, 1024, 16
    E = _rand(Q, Q, seed=13).to(DEV, torch.bfloat16)
    Wp = _rand(FS, D, Q, seed=14).to(DEV, torch.bfloat16)
    out = torch.empty((FS, Q, D), device=DEV, dtype=out_dtype)
    n0 = hip.lib().dll.srnn_blaslt_calls()
    hip.gemm(E, Wp, transB=True, out=out, out_dtype=out_dtype, M=Q, N=D, K=Q, lda=Q, ldb=Q,
             ldc=D, batch=FS, sA=0, sB=D * Q, sC=Q * D)
    torch.cuda.synchronize()
    assert hip.lib().dll.srnn_blaslt_calls() - n0 == 1
    ref = torch.einsum('qj,kdj->kqd', E.float().cpu(), Wp.float().cpu())
    tol = 2e-3 * np.sqrt(Q) if out_dtype == torch.float32 else 1e-2 * np.sqrt(Q)
    torch.testing.assert_close(out.float().cpu(), ref, atol=tol, rtol=1e-2)


@pytest.mark.parametrize('src_dt,dst_dt', [(torch.float32, torch.bfloat16),
                                           (torch.float32, torch.float32),
                                           (torch.bfloat16, torch.float32),
                                           (torch.bfloat16, torch.bfloat16)])
@pytest.mark.parametrize('rows,cols', [(1, 1), (1, 7), (3, 5), (131072, 43), (4097, 1024)])
def test_cast_dense_and_strided(hip, src_dt, dst_dt, rows, cols):
    """srnn_copy2d: the dense four-per-lane path (with its scalar tail) and the strided
    element path both give torch's round-to-nearest-even conversion bit for bit."""
    x = (_rand(rows, cols, seed=rows + cols) * 3.0).to(DEV, src_dt)
    x[0, 0] = float('nan') if src_dt == torch.float32 else x[0, 0]
    got = torch.empty((rows, cols), device=DEV, dtype=dst_dt)
    hip.lib().call('srnn_copy2d', hip.dcode(x), hip.dcode(got), rows, cols, hip.ptr(x), cols,
                   hip.ptr(got), cols, hip.stream())
    want = x.to(dst_dt)
    assert got.shape == want.shape
    assert torch.equal(got.view(-1).float().nan_to_num(7.0), want.view(-1).float().nan_to_num(7.0))
    # strided source and destination (a column window of wider rows): the element path
    if cols > 1:
        src = torch.zeros((rows, cols + 3), device=DEV, dtype=src_dt)
        src[:, 1:cols + 1] = x
        dst = torch.full((rows, cols + 5), -1.0, device=DEV, dtype=dst_dt)
        hip.lib().call('srnn_copy2d', hip.dcode(src), hip.dcode(dst), rows, cols - 1,
                       hip.ptr(src[:, 1:]), cols + 3, hip.ptr(dst[:, 2:]), cols + 5, hip.stream())
        assert torch.equal(dst[:, 2:cols + 1].float().nan_to_num(7.0),
                           x[:, :cols - 1].to(dst_dt).float().nan_to_num(7.0))
        assert bool((dst[:, :2] == -1).all()) and bool((dst[:, cols + 1:] == -1).all())
