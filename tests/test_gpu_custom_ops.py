"""The HIP operators as registered torch.library custom ops (custom_ops.py).

* torch.library.opcheck on every op with real inputs: schema (declared mutations only),
  fake-kernel agreement, autograd registration and the AOT-dispatch round trip;
* the drop-in Predictor's forward under torch.compile (fullgraph=False, eager backend: no
  Triton on this image) traces without a graph break inside the ops and gives the eager
  log-probs bit for bit.
"""
import numpy as np
import pytest
import torch

import recipe

pytestmark = pytest.mark.gpu
DEV = 'cuda'
# opcheck's utilities (test_aot_dispatch_dynamic runs the op through AOT autograd)
UTILS = ('test_schema', 'test_autograd_registration', 'test_faketensor',
         'test_aot_dispatch_dynamic')


def _model(dtype=torch.float32, cfg='t3', seed=3):
    import model as M
    c = recipe.CONFIGS[cfg]
    m = M.SampleRNN(c['frame_sizes'], c['n_rnn'], c['dim'], c['learn_h0'], c['q_levels'], True,
                    c['weight_norm'], c['cond_dim'], c['spk_dim'])
    m.compute_dtype = dtype
    pred = M.Predictor(m)
    pred.load_state_dict({k: torch.from_numpy(v.copy())
                          for k, v in recipe.make_weights(c, seed).items()})
    return m.to(DEV), pred.to(DEV), c


def _batch(c, B=2, T=128, seed=4):
    L = int(np.prod(c['frame_sizes']))
    g = torch.Generator().manual_seed(seed)
    x = torch.randint(0, 256, (B, L + T), generator=g).to(DEV)
    cond = torch.rand(B, T // L, c['cond_dim'], generator=g, dtype=torch.float64).to(DEV)
    spk = (torch.arange(B) % c['spk_dim']).reshape(-1, 1).to(DEV)
    return x, cond, spk, L


def test_every_op_registered(hip):
    import custom_ops
    for name in custom_ops.OPS:
        assert hasattr(torch.ops.srnn, name), name


@pytest.mark.parametrize('cfg,dtype', [('t3', torch.float32), ('t3r2wn', torch.float32),
                                       ('t3', torch.bfloat16)])
def test_opcheck_tier_and_mlp(hip, cfg, dtype):
    import model as M
    import utils
    m, pred, c = _model(dtype, cfg)
    x, cond, spk, L = _batch(c)
    top, bot = m.frame_level_rnns[-1], m.frame_level_rnns[0]
    B = x.shape[0]
    n = top.n_frame_samples
    prev = utils._dequant(x[:, L - n: x.shape[1] - n], 256, 2.0).view(B, -1, n)
    args = (prev.float().contiguous(), None, cond, spk, None, top.h0, top._param_list(),
            M.tier_meta(top))
    torch.library.opcheck(torch.ops.srnn.tier_fwd.default, args, test_utils=UTILS)
    upper, _ = top(prev, None, None, cond, spk, None, None)
    n = bot.n_frame_samples
    prevb = utils._dequant(x[:, L - n: x.shape[1] - n], 256, 2.0).view(B, -1, n)
    args = (prevb.float().contiguous(), upper.detach().contiguous().requires_grad_(True), None,
            None, None, bot.h0, bot._param_list(), M.tier_meta(bot))
    torch.library.opcheck(torch.ops.srnn.tier_fwd.default, args, test_utils=UTILS)
    u, _ = bot(prevb, upper, None, None, None, None, None)
    mlp = m.sample_level_mlp
    fs0 = mlp.frame_size
    xi = x[:, L - fs0: x.shape[1] - 1].contiguous()
    args = (xi, u.detach().contiguous().requires_grad_(True), mlp._param_list(),
            M.mlp_meta(mlp))
    torch.library.opcheck(torch.ops.srnn.mlp_fwd.default, args, test_utils=UTILS)


def test_opcheck_nll_upsample_dequant(hip):
    import nn as snn
    g = torch.Generator().manual_seed(1)
    lp = torch.log_softmax(torch.randn(2, 64, 256, generator=g), -1).to(DEV).requires_grad_(True)
    tgt = torch.randint(0, 256, (2, 64), generator=g).to(DEV)
    torch.library.opcheck(torch.ops.srnn.nll_bits.default, (lp, tgt), test_utils=UTILS)
    up = snn.LearnedUpsampling1d(32, 48, 4).to(DEV)
    snn.apply_weight_norm(up.conv_t)
    up = up.to(DEV)
    xx = torch.randn(3, 32, 7, generator=g).to(DEV).requires_grad_(True)
    params = [up.conv_t.weight_g, up.conv_t.weight_v, up.bias]
    torch.library.opcheck(torch.ops.srnn.upsample.default, (xx, params, 4, True, True),
                          test_utils=UTILS)
    idx = torch.randint(0, 256, (3, 40), generator=g).to(DEV)
    torch.library.opcheck(torch.ops.srnn.dequant.default, (idx, 256, 2.0, 0),
                          test_utils=('test_schema', 'test_faketensor'))


def test_opcheck_adam_and_generate(hip):
    import model as M
    g = torch.Generator().manual_seed(2)
    ps = [torch.randn(37, generator=g).to(DEV), torch.randn(4, 64, generator=g).to(DEV)]
    gs = [torch.randn(37, generator=g).to(DEV) * 3, None]
    ms = [torch.zeros_like(p) for p in ps]
    vs = [torch.zeros_like(p) for p in ps]
    sh = [None, torch.empty(4, 64, device=DEV, dtype=torch.bfloat16)]
    torch.library.opcheck(torch.ops.srnn.adam_clip_.default,
                          (ps, gs, ms, vs, sh, 1.0, -1.0, 1.0, 1e-3, 0.9, 0.999, 1e-8, 1),
                          test_utils=('test_schema', 'test_faketensor'))
    m, _, c = _model(torch.float32, 't3')
    weights, meta = M.generation_weights(m)
    cond = torch.rand(2, 2, c['cond_dim'], generator=g).to(DEV)
    rb = M.top_row_bias(m, torch.tensor([1, 2], device=DEV))
    torch.library.opcheck(torch.ops.srnn.generate.default,
                          (weights, meta, cond, rb, None, 7, 0, 1, True),
                          test_utils=('test_schema', 'test_faketensor'))


def test_predictor_forward_compiles_without_leaving_the_ops(hip):
    import torch._dynamo as dynamo
    m, pred, c = _model(torch.float32, 't3')
    x, cond, spk, L = _batch(c)
    with torch.no_grad():
        ref = pred(x[:, :-1], True, cond, spk)
        pred.reset_hidden_states()
        dynamo.reset()
        expl = dynamo.explain(pred.forward)(x[:, :-1], True, cond, spk)
        assert expl.graph_break_count == 0, expl.break_reasons
        ops = {str(n.target) for gm in expl.graphs for n in gm.graph.nodes
               if n.op == 'call_function'}
        assert any('srnn.tier_fwd' in o for o in ops) and any('srnn.mlp_fwd' in o for o in ops)
        dynamo.reset()
        pred.reset_hidden_states()
        comp = torch.compile(pred.forward, backend='eager', fullgraph=False)
        out = comp(x[:, :-1], True, cond, spk)
    assert torch.equal(out, ref)
