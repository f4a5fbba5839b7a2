"""Model-level parity of the HIP path (drop-in model.py / Trainer) with the reference.

Goldens (tests/golden/*.npz) were produced by running the reference itself; weights and
inputs are regenerated from the seeded recipe.  Tolerances: fp32 logits/log-probs 1e-4
(north star), sample indices bit-exact, TBPTT losses 1e-4.
"""
import numpy as np
import pytest
import torch

import recipe
from conftest import golden

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def build(cfg, weights, dtype=torch.float32):
    import model as M
    m = M.SampleRNN(cfg['frame_sizes'], cfg['n_rnn'], cfg['dim'], cfg['learn_h0'],
                    cfg['q_levels'], True, cfg['weight_norm'], cfg['cond_dim'], cfg['spk_dim'])
    m.compute_dtype = dtype
    pred = M.Predictor(m)
    sd = {k: torch.from_numpy(v.copy()) for k, v in weights.items()}
    pred.load_state_dict(sd, strict=True)
    return m.to(DEV), pred.to(DEV)


@pytest.mark.parametrize('name', ['t2', 't3', 't3r2wn', 't4la', 't3_20_4', 'big', 'a', 'e'])
def test_forward_golden(hip, name):
    g = golden('fwd_' + name)
    cfg = recipe.CONFIGS[name]
    m, pred = build(cfg, recipe.make_weights(cfg, int(g['weight_seed'])))
    with torch.no_grad():
        for n in range(int(g['n_chunks'])):
            lp = pred(torch.from_numpy(g['input_%d' % n]), bool(g['reset_%d' % n]),
                      torch.from_numpy(g['cond_%d' % n]), torch.from_numpy(g['spk_%d' % n]))
            lp = lp.cpu().numpy()
            if 'keep_rows' in g:
                np.testing.assert_allclose(lp[:, g['keep_rows']], g['logp_rows_%d' % n],
                                           atol=1e-4, rtol=0)
                np.testing.assert_allclose(lp.astype(np.float64).sum(axis=(1, 2)),
                                           g['logp_sum_%d' % n], rtol=1e-5)
            else:
                np.testing.assert_allclose(lp, g['logp_%d' % n], atol=1e-4, rtol=0)
            for t, rnn in enumerate(m.frame_level_rnns):
                np.testing.assert_allclose(pred.hidden_states[rnn].cpu().numpy(),
                                           g['hidden_%d_tier%d' % (n, t)], atol=2e-5, rtol=0)


@pytest.mark.parametrize('name', ['t2', 't3', 't4la', 't3_20_4', 't3r2wn', 'big', 'a', 'e'])
@pytest.mark.parametrize('graph,persistent', [(True, True), (False, True), (True, False),
                                              (False, False)])
def test_generation_golden(hip, name, graph, persistent):
    """fp32 generation with the reference's replayed multinomial noise: index streams bit
    for bit, log-probs 1e-4 ('big' = configs[2]'s dim-1024 model, 128 samples; 'e' =
    configs[4]'s 4-tier dim-1024 look-ahead model, FS [16, 4, 4], 512 samples)."""
    import model as M
    g = golden('gen_' + name)
    cfg = recipe.CONFIGS[name]
    m, _ = build(cfg, recipe.make_weights(cfg, int(g['weight_seed'])))
    gen = M.Generator(m, True)
    out, lp = gen(int(g['n_seqs']), 0, g['cond'], int(g['spk']), noise=g['noise'],
                  return_logp=True, use_graph=graph, persistent=persistent)
    L = m.lookback
    idx = gen.last_sequences[:, L:].cpu().numpy()
    assert np.array_equal(idx, g['idx'])
    assert np.array_equal(out.numpy(), g['samples'])
    np.testing.assert_allclose(lp.cpu().numpy(), g['logp'], atol=1e-4, rtol=0)


@pytest.mark.parametrize('name', ['t3', 'big'])
def test_generation_default_sampler_from_seed(hip, name):
    """The default path exactly as generate.py drives it (generate.py:200-253): seed, build
    the model (its init consumes the CPU generator in the reference's order, a13), load the
    weights, call the Generator with no noise= argument -- sampler='torch' draws the
    multinomials' Exp(1) noise from torch's CPU generator in the reference's consumption
    order.  The index stream equals the one the reference produced from the same seed."""
    import model as M
    g = golden('genseed_' + name)
    cfg = recipe.CONFIGS[name]
    torch.manual_seed(int(g['gen_seed']))
    m = M.SampleRNN(cfg['frame_sizes'], cfg['n_rnn'], cfg['dim'], cfg['learn_h0'],
                    cfg['q_levels'], True, cfg['weight_norm'], cfg['cond_dim'], cfg['spk_dim'])
    pred = M.Predictor(m)
    w = recipe.make_weights(cfg, int(g['weight_seed']))
    pred.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in w.items()}, strict=True)
    m = m.to(DEV)
    gen = M.Generator(m, True)
    out = gen(int(g['n_seqs']), 0, g['cond'], int(g['spk']))
    assert np.array_equal(gen.last_sequences[:, m.lookback:].cpu().numpy(), g['idx'])
    assert np.array_equal(out.numpy(), g['samples'])


class _GradCapture:
    trigger_interval = [(1, 'iteration')]

    def __init__(self, pred):
        self.pred = pred
        self.grads = []

    def register(self, trainer):
        self.trainer = trainer

    def iteration(self, *args):
        self.grads.append({k: (p.grad.detach().cpu().numpy().copy() if p.grad is not None
                               else np.zeros(tuple(p.shape), np.float32))
                           for k, p in self.pred.named_parameters()})


@pytest.mark.parametrize('name', ['t3', 't3r2wn', 't2'])
def test_tbptt_golden(hip, name):
    import nn as snn
    import optim
    from trainer import Trainer
    g = golden('tbptt_' + name)
    cfg = recipe.CONFIGS[name]
    m, pred = build(cfg, recipe.make_weights(cfg, int(g['weight_seed'])))
    B = int(g['B'])
    opt = optim.gradient_clipping(torch.optim.Adam(pred.parameters(), lr=float(g['lr'])))
    losses = []

    def criterion(out, tgt):
        loss = snn.sequence_nll_loss_bits(out, tgt)
        losses.append(float(loss.detach()))
        return loss
    data = [(torch.from_numpy(g['input_%d' % s]), torch.tensor([int(g['reset_%d' % s])] * B),
             torch.from_numpy(g['target_%d' % s]), torch.from_numpy(g['cond_%d' % s]),
             torch.from_numpy(g['spk_%d' % s])) for s in range(int(g['n_steps']))]
    tr = Trainer(pred, criterion, opt, data, True, None)
    cap = _GradCapture(pred)
    tr.register_plugin(cap)
    tr.run(1)
    np.testing.assert_allclose(losses, g['losses'], atol=1e-4, rtol=0)
    names = [str(s) for s in g['names']]
    for s in range(2):
        for k in names:
            np.testing.assert_allclose(cap.grads[s][k], g['grad_%d/%s' % (s, k)], atol=1e-4,
                                       rtol=1e-3, err_msg='step %d %s' % (s, k))
    params = dict(pred.named_parameters())
    for k in names:
        np.testing.assert_allclose(params[k].detach().cpu().numpy(), g['param_final/' + k],
                                   atol=2e-4, rtol=0, err_msg=k)


def test_generation_vs_oracle_philox_consistency(hip):
    """Device-RNG sampling: the teacher-forced Predictor on the generated stream must give
    the per-step log-probs the generator sampled from (SURVEY §3.3 invariant)."""
    import model as M
    cfg = recipe.CONFIGS['t3']
    m, pred = build(cfg, recipe.make_weights(cfg, 41))
    n_seqs, num_cond = 4, 6
    cond = recipe.synth_cond((n_seqs, num_cond, cfg['cond_dim']), 3)
    spk = np.arange(n_seqs) % cfg['spk_dim']
    gen = M.Generator(m, True)
    _, lp = gen(n_seqs, 0, cond, spk, sampler='philox', seed=1234, return_logp=True)
    seq = gen.last_sequences
    L = m.lookback
    with torch.no_grad():
        tf = pred(seq[:, :-1], True, torch.from_numpy(cond), torch.from_numpy(spk).reshape(-1, 1))
    torch.testing.assert_close(tf.cpu(), lp.cpu(), atol=1e-4, rtol=0)
    # sampled indices follow the distribution: mean log-prob of the drawn samples is finite
    assert torch.isfinite(lp).all()


def test_mask_bits_step_bf16(hip, monkeypatch):
    """SRNN_MASK_BITS=1 (ReLU masks of a1 / a2 kept as bits for the backward): the bf16
    forward log-probs and every gradient equal the default path's bit for bit."""
    import nn as snn
    cfg = dict(recipe.CONFIGS['t3'], dim=256)
    B, T = 4, 1024
    g = torch.Generator().manual_seed(3)
    outs = []
    for flag in ('0', '1'):
        monkeypatch.setenv('SRNN_MASK_BITS', flag)
        m, pred = build(cfg, recipe.make_weights(cfg, 21), torch.bfloat16)
        L = m.lookback
        g.manual_seed(3)
        x = torch.randint(0, 256, (B, L + T), generator=g)
        cond = torch.rand(B, T // L, cfg['cond_dim'], generator=g)
        spk = torch.arange(B).reshape(-1, 1) % cfg['spk_dim']
        lp = pred(x[:, :-1].to(DEV), True, cond, spk)
        loss = snn.sequence_nll_loss_bits(lp, x[:, L:].to(DEV))
        loss.backward()
        outs.append((lp.detach().cpu(), {k: p.grad.detach().cpu().clone()
                                          for k, p in pred.named_parameters()
                                          if p.grad is not None}))
    assert torch.equal(outs[0][0], outs[1][0])
    assert outs[0][1].keys() == outs[1][1].keys()
    for k in outs[0][1]:
        assert torch.equal(outs[0][1][k], outs[1][1][k]), k


def test_a1_bits_step_bf16(hip, monkeypatch):
    """The default grouped a1 mask bits (SRNN_A1_BITS=1: the L1 kernel writes them, the da1
    GEMM stages them by LDS-DMA): log-probs and every gradient equal the bf16-mask path's
    (SRNN_A1_BITS=0) bit for bit, at D = 1024 (the pair-mode kernel's grouped-bits form)."""
    import nn as snn
    cfg = dict(recipe.CONFIGS['t3'], dim=1024)
    B, T = 8, 1024
    g = torch.Generator().manual_seed(5)
    outs = []
    for flag in ('0', '1'):
        monkeypatch.setenv('SRNN_A1_BITS', flag)
        m, pred = build(cfg, recipe.make_weights(cfg, 23), torch.bfloat16)
        L = m.lookback
        g.manual_seed(5)
        x = torch.randint(0, 256, (B, L + T), generator=g)
        cond = torch.rand(B, T // L, cfg['cond_dim'], generator=g)
        spk = torch.arange(B).reshape(-1, 1) % cfg['spk_dim']
        lp = pred(x[:, :-1].to(DEV), True, cond, spk)
        loss = snn.sequence_nll_loss_bits(lp, x[:, L:].to(DEV))
        loss.backward()
        outs.append((lp.detach().cpu(), {k: p.grad.detach().cpu().clone()
                                          for k, p in pred.named_parameters()
                                          if p.grad is not None}))
    assert torch.equal(outs[0][0], outs[1][0])
    assert outs[0][1].keys() == outs[1][1].keys()
    for k in outs[0][1]:
        assert torch.equal(outs[0][1][k], outs[1][1][k]), k
