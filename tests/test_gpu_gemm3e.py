"""gemm3e (the 8-phase ping-pong NT kernel, csrc/gemm3.hip) == the pair-mode gemm3p kernel bit
for bit: the same MFMA k order per output fragment, so switching kernels must not change a
single output bit (bf16 / fp32 outputs, bias, ReLU, ReLU bits out, alpha), for one tile, one
round of tiles, several tiles per workgroup and a ragged last round.  Both are also held to a
torch fp32 reference.  These are the GEMMs of model.py:287-301 (SampleLevelMLP layers) and
nn.py:33-43 (LearnedUpsampling1d) in their forward NT layout."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = 'cuda'


def _rand(*shape, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(*shape, generator=g) * 2 - 1


SHAPES = [(256, 256, 128), (512, 768, 192), (8192, 512, 1024), (65536, 1024, 256),
          (256 * 37, 256 * 9, 320), (4096, 3072, 128)]


def _run(hip, monkeypatch, g3e, a, w, **kw):
    monkeypatch.setenv('SRNN_BLASLT', '0')
    monkeypatch.setenv('SRNN_G3E', '1' if g3e else '0')
    out = hip.gemm(a, w, transB=True, **kw)
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize('M,N,K', SHAPES)
@pytest.mark.parametrize('kind', ['bf16_bias_relu_bits', 'bf16_plain', 'fp32_bias', 'bf16_alpha'])
def test_gemm3e_equals_pair_mode(hip, monkeypatch, M, N, K, kind):
    bf = torch.bfloat16
    a = _rand(M, K, seed=1).to(DEV, bf)
    w = _rand(N, K, seed=2).to(DEV, bf)
    bias = (_rand(N, seed=3) * 0.5).to(DEV)
    kw = {}
    if kind == 'bf16_bias_relu_bits':
        kw = dict(out_dtype=bf, bias=bias, relu=True)
    elif kind == 'bf16_plain':
        kw = dict(out_dtype=bf)
    elif kind == 'fp32_bias':
        kw = dict(out_dtype=torch.float32, bias=bias)
    else:
        kw = dict(out_dtype=bf, alpha=0.37, bias=bias)
    res = []
    for g3e in (False, True):
        bits = hip.relu_bits(M, N, DEV) if kind == 'bf16_bias_relu_bits' else None
        o = _run(hip, monkeypatch, g3e, a, w, bits_out=bits, **kw)
        res.append((o, bits))
    assert torch.equal(res[0][0], res[1][0])
    if res[0][1] is not None:
        assert torch.equal(res[0][1], res[1][1])
    # both against a torch fp32 product (a sample of rows for the big shapes)
    rows = torch.arange(0, M, max(1, M // 512), device=DEV)
    ref = a[rows].float() @ w.float().t()
    ref = ref * kw.get('alpha', 1.0)
    if 'bias' in kw:
        ref = ref + bias
    if kw.get('relu'):
        ref = ref.clamp_min(0)
    tol = 2e-3 * np.sqrt(K) + (0.02 if kw['out_dtype'] == bf else 0.0) * ref.abs().max().item()
    torch.testing.assert_close(res[1][0][rows].float(), ref, atol=tol, rtol=1e-2)
    if res[1][1] is not None:
        # the bits are those of the stored bf16 values (> 0)
        st = res[1][0][rows].float() > 0
        bits = res[1][1][rows].to(torch.int32) & 0xffff
        cols = torch.arange(N, device=DEV)
        got = ((bits[:, cols // 16] >> (cols % 16)) & 1).bool()
        assert torch.equal(got, st)


def test_gemm3e_k64_takes_pair_mode(hip, monkeypatch):
    """K = 64 (one k-tile per output tile) is not admitted to gemm3e (its bias buffers need
    two k-tiles per tile): the call runs on the pair mode and matches it."""
    bf = torch.bfloat16
    a = _rand(4096, 64, seed=4).to(DEV, bf)
    w = _rand(512, 64, seed=5).to(DEV, bf)
    bias = _rand(512, seed=6).to(DEV)
    o0 = _run(hip, monkeypatch, False, a, w, out_dtype=bf, bias=bias, relu=True)
    o1 = _run(hip, monkeypatch, True, a, w, out_dtype=bf, bias=bias, relu=True)
    assert torch.equal(o0, o1)


@pytest.mark.parametrize('M', [32768, 131072])
def test_logits_gemm_logsoftmax_epilogue(hip, M):
    """srnn_gemm_logsoftmax_next: the logits GEMM (bf16 a2 (M, 1024) . W_out^T (256, 1024) +
    bias, fp32 out) writes log_softmax of its rows (model.py:324-325) -- against torch's
    log_softmax of the fp32 product and against the unfused path (fp32 logits, then
    srnn_logsoftmax_nll); several tiles per workgroup at M = 131072."""
    bf = torch.bfloat16
    a = (_rand(M, 1024, seed=7) * 2).to(DEV, bf)
    w = (_rand(256, 1024, seed=8) * 0.2).to(DEV, bf)
    b = _rand(256, seed=9).to(DEV)
    lib = hip.lib().dll
    lib.srnn_gemm_logsoftmax_next()
    lp = hip.linear(a, w, bias=b)
    assert lib.srnn_gemm_logsoftmax_taken() == 1
    z = hip.linear(a, w, bias=b)                              # plain logits (no request)
    assert lib.srnn_gemm_logsoftmax_taken() == 0
    lp2 = torch.empty_like(z)
    hip.lib().call('srnn_logsoftmax_nll', hip.ptr(z), 256, None, 0, M, M, 256, None,
                   hip.ptr(lp2), 256, None, hip.F32, 0, 0.0, hip.stream())
    torch.cuda.synchronize()
    rows = torch.arange(0, M, max(1, M // 1024), device=DEV)
    ref = torch.log_softmax(a[rows].double() @ w.double().t() + b.double(), dim=1)
    assert (lp[rows].double() - ref).abs().max().item() < 5e-5
    assert (lp - lp2).abs().max().item() < 1e-5


@pytest.mark.parametrize('M', [300, 4096])
def test_logsoftmax_request_not_taken_falls_back(hip, M):
    """Shapes the epilogue does not take (M not a multiple of 256; too few 256-row tiles for
    the gemm3 path): the request is not taken, the GEMM writes plain logits, and taken()
    clears the request."""
    bf = torch.bfloat16
    a = _rand(M, 1024, seed=10).to(DEV, bf)
    w = _rand(256, 1024, seed=11).to(DEV, bf)
    lib = hip.lib().dll
    lib.srnn_gemm_logsoftmax_next()
    z = hip.linear(a, w)
    assert lib.srnn_gemm_logsoftmax_taken() == 0
    torch.cuda.synchronize()
    ref = a.float() @ w.float().t()
    torch.testing.assert_close(z, ref, atol=2e-3 * 32, rtol=1e-2)
