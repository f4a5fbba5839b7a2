"""Round 4: parity at the MEASURED dimensions, pinned to the reference itself.

Fixtures (tests/golden/make_golden.py --only big4, produced by running the reference):
  * tbptt_big -- configs[1]'s model (3-tier FS [16, 4], D = 1024, C = 43, 6 speakers), B = 2,
    T = 1024, 3 chunks through the reference's Trainer (reset, then carried state; clip +
    Adam): losses, hidden state after every chunk, and per tensor a sum / L2 norm / seeded
    4096-entry sample of the gradients of every chunk and of the final parameters;
  * tbptt_a -- the same for configs[0] (2-tier FS [16], D = 256, one speaker);
  * fwd_a / gen_a -- configs[0]'s forward log-probs and a generation index stream;
  * genlong_big -- 2 rows x 75 top-tier frames = 4,800 samples of configs[2]'s model with
    the reference's multinomial noise replayed.
Tolerances: every TBPTT quantity within 3x the reference's own distance when its initial
weights are perturbed by one ulp (conftest.within_floor: at D = 1024 rounding flips a few
ReLU masks and Adam's sign-driven first steps amplify it -- the reference moves 0.04-0.12
in the chunk-2 hidden state and 2e-4 in the loss) plus the strict tolerance (losses 1e-4,
gradients 1e-4 + 1e-3 max |g|, parameters 2e-4); indices bit-exact; log-probs 1e-4.

Two checks of the measured paths without a reference fixture:
  * bf16 TBPTT loss trajectory: 50 chunks at B = 128 (configs[1]) in bf16 and in fp32 from
    the same weights and data; the per-chunk loss difference is bounded against the bf16
    path's own one-ulp sensitivity (bound in the test);
  * fp32 persistent generation over 750 top-tier ticks at B = 128 (configs[2], 48,000
    samples): every log-prob the loop sampled from equals the teacher-forced fp32
    Predictor's on the generated stream within 1e-4 (SURVEY §3.3 invariant).
"""
import numpy as np
import pytest
import torch

import recipe
from conftest import golden, genlong_noise, within_floor, within_floor_sampled

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def build(cfg, weights, dtype=torch.float32):
    import model as M
    m = M.SampleRNN(cfg['frame_sizes'], cfg['n_rnn'], cfg['dim'], cfg['learn_h0'],
                    cfg['q_levels'], True, cfg['weight_norm'], cfg['cond_dim'], cfg['spk_dim'])
    m.compute_dtype = dtype
    pred = M.Predictor(m)
    pred.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in weights.items()},
                         strict=True)
    return m.to(DEV), pred.to(DEV)


class _Capture:
    """Iteration plugin: every chunk's clamped gradients and the carried hidden state."""
    trigger_interval = [(1, 'iteration')]

    def __init__(self, pred, model):
        self.pred, self.model = pred, model
        self.grads, self.hidden = [], []

    def register(self, trainer):
        self.trainer = trainer

    def iteration(self, *args):
        self.grads.append({k: (p.grad.detach().cpu().numpy().copy() if p.grad is not None
                               else np.zeros(tuple(p.shape), np.float32))
                           for k, p in self.pred.named_parameters()})
        self.hidden.append([self.pred.hidden_states[r].detach().cpu().numpy().copy()
                            for r in self.model.frame_level_rnns])


@pytest.mark.parametrize('name', ['big', 'a'])
def test_tbptt_sampled_golden(hip, name):
    """fp32 HIP TBPTT (3 chunks through the drop-in Trainer, graph mode from the 3rd) against
    the reference's trajectory: losses, hidden states after every chunk, every chunk's
    gradients and the final parameters within FLOOR x the reference's own distance under a
    one-ulp weight perturbations (conftest.within_floor) plus the strict tolerances (losses
    1e-4, hidden 2e-5, gradients 1e-4 + 1e-3 max|g|, parameters 2e-4)."""
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
    n_steps = int(g['n_steps'])
    data = [(torch.from_numpy(g['input_%d' % s]), torch.tensor([int(g['reset_%d' % s])] * B),
             torch.from_numpy(g['target_%d' % s]), torch.from_numpy(g['cond_%d' % s]),
             torch.from_numpy(g['spk_%d' % s])) for s in range(n_steps)]
    tr = Trainer(pred, criterion, opt, data, True, None)
    cap = _Capture(pred, m)
    tr.register_plugin(cap)
    tr.run(1)
    names = [str(s) for s in g['names']]
    fails = []

    def check(fn, *a, **k):
        try:
            fn(*a, **k)
        except AssertionError as e:
            fails.append(str(e).strip().splitlines()[0][:200])
    print('losses', losses, 'reference', list(g['losses']), 'perturbation envelope %.3g'
          % float(g['env_max/losses']))
    # chunk 0 (fresh weights: the forward + backward proper, before any Adam step) is held
    # to the strict 1e-4 alone -- the perturbed reference moves it by ~1e-7; the envelope
    # (whose 'losses' key is the max over chunks, set by chunk 2) covers the later chunks only
    check(np.testing.assert_allclose, losses[0], g['losses'][0], atol=1e-4, rtol=0,
          err_msg='chunk-0 loss')
    check(within_floor, losses[1:], g['losses'][1:], g, 'losses', 1e-4)
    for s in range(n_steps):
        for t in range(len(cfg['frame_sizes'])):
            key = 'hidden_%d_tier%d' % (s, t)
            r = g[key]
            print('chunk %d tier %d hidden max |diff| %.3g (perturbation envelope %.3g)' % (
                s, t, np.abs(cap.hidden[s][t] - r).max(), float(g['env_max/' + key])))
            check(within_floor, cap.hidden[s][t], r, g, key, 2e-5)
        for k in names:
            check(within_floor_sampled, cap.grads[s][k], g, 'grad_%d' % s, k, 1e-4, 1e-3)
    params = dict(pred.named_parameters())
    for k in names:
        check(within_floor_sampled, params[k].detach().cpu().numpy(), g, 'param_final', k, 2e-4)
    for f in fails:
        print('FAIL', f)
    assert not fails, '%d checks failed (first: %s)' % (len(fails), fails[0])


@pytest.mark.parametrize('graph,persistent', [(True, True), (False, True), (True, False)])
def test_generation_long_golden(hip, graph, persistent):
    """4,800 samples (75 top-tier ticks, 300 bottom ticks) of configs[2]'s model in fp32:
    the index stream equals the reference's bit for bit, log-probs at every 16th step 1e-4."""
    import model as M
    g = golden('genlong_big')
    cfg = recipe.CONFIGS['big']
    q = genlong_noise(g)
    m, _ = build(cfg, recipe.make_weights(cfg, int(g['weight_seed'])))
    gen = M.Generator(m, True)
    out, lp = gen(int(g['n_seqs']), 0, g['cond'], int(g['spk']), noise=q, return_logp=True,
                  use_graph=graph, persistent=persistent)
    L = m.lookback
    idx = gen.last_sequences[:, L:].cpu().numpy()
    ref = g['idx'].astype(np.int64)
    mism = np.argwhere(idx != ref)
    assert mism.size == 0, 'first mismatch (row, step) %s of %d' % (mism[:1], mism.shape[0])
    lut = golden('ulaw')['lut']
    assert np.array_equal(out.numpy(), lut[ref])
    np.testing.assert_allclose(lp.cpu().numpy()[:, g['logp_steps']], g['logp'], atol=1e-4,
                               rtol=0)


def test_bf16_loss_trajectory_50_chunks(hip):
    """configs[1] (B = 128, T = 1024): 50 TBPTT chunks (reset, then 49 carried) with clip +
    Adam from the same weights and data in bf16 (the bench's path) and in fp32 (the path
    pinned to the reference).  Over 50 Adam steps a rounding-level change moves the
    trajectory by itself (sign-driven first moments of near-zero gradients).  Fixed bounds,
    set from the round-4 measurements on MI355X: max relative loss difference 2.7e-3 .. 5.7e-3
    (chunk 35 / 43, depending on the summation order of one bias gradient), mean 6.8e-4 ..
    9.3e-4, and the bf16 run's own one-ulp-perturbation sensitivity up to 5.1e-3
    (profiles/r04_traj_50chunks.log).  Round 6 re-measured the envelope with the log-softmax
    epilogue on and off and from two one-ulp weight perturbations (tools/traj_env.py,
    profiles/r06_traj_envelope.txt): max 8.5e-3 (epilogue on), 5.7e-3 (off), 4.3e-3 and 8.9e-3
    (perturbed), means 8.1e-4 .. 1.28e-3 -- a one-ulp change of the initial weights alone
    reaches 8.9e-3, so the bound is 1.5e-2 on every chunk (1.7x the largest rounding-level
    excursion), the mean below 1.5e-3, chunk 0 (no Adam step yet) within 1e-3; DESIGN §4."""
    import bench
    import nn as snn
    import optim
    B, T, L, N = 128, 1024, 64, 50
    batches = bench.gpu_batches(bench.synth_batches(B, T, L, N, 0), DEV)

    def traj(dtype):
        _, pred = bench.make_model(dtype)
        pred = pred.to(DEV)
        opt = optim.gradient_clipping(torch.optim.Adam(pred.parameters(), lr=1e-3))
        out = []
        for inp, reset, tgt, cnd, spk in batches:
            opt.zero_grad()

            def closure():
                loss = snn.sequence_nll_loss_bits(pred(inp, reset, cnd, spk), tgt)
                loss.backward()
                return loss
            out.append(opt.step(closure).detach())
        import samplernn_hip as H
        H.check_persistent_errors()
        return torch.stack(out).double().cpu().numpy()
    b = traj(torch.float32)
    a = traj(torch.bfloat16)
    rel = np.abs(a - b) / np.abs(b)
    print('bf16-vs-fp32 loss trajectory over %d chunks: max rel %.3g (chunk %d), mean rel %.3g;'
          ' fp32 %.4f -> %.4f, bf16 %.4f -> %.4f'
          % (N, rel.max(), int(rel.argmax()), rel.mean(), b[0], b[-1], a[0], a[-1]))
    assert np.all(np.isfinite(a))
    assert rel[0] < 1e-3
    assert rel.max() < 1.5e-2 and rel.mean() < 1.5e-3


def test_persistent_fp32_long_teacher_forced(hip):
    """configs[2] in fp32: B = 128 rows x 750 top-tier ticks (48,000 samples) through the
    persistent loop (Philox draws); the teacher-forced fp32 Predictor over the generated
    stream (50 chunks of 960 samples, hidden state carried) reproduces every log-prob the
    loop sampled from within 1e-4."""
    import model as M
    cfg = recipe.CONFIGS['big']
    m, pred = build(cfg, recipe.make_weights(cfg, 77977))
    B, num_cond = 128, 750
    L = m.lookback
    cond = recipe.synth_cond((B, num_cond, cfg['cond_dim']), 1)
    spk = np.arange(B) % cfg['spk_dim']
    gen = M.Generator(m, True)
    _, lp = gen(B, 0, cond, spk, sampler='philox', seed=5, return_logp=True)
    seq = gen.last_sequences                         # (B, L + T) on the device
    lp = lp.to(DEV) if lp.device.type != 'cuda' else lp
    T = num_cond * L
    C = 960
    condt = torch.from_numpy(cond)
    spkt = torch.from_numpy(spk).reshape(-1, 1)
    worst = 0.0
    with torch.no_grad():
        for n in range(T // C):
            x = seq[:, n * C: n * C + L + C - 1]
            tf = pred(x, n == 0, condt[:, n * C // L:(n + 1) * C // L], spkt)
            d = (tf - lp[:, n * C:(n + 1) * C]).abs().max().item()
            worst = max(worst, d)
    print('persistent fp32 vs teacher-forced over %d samples x %d rows: max |dlogp| %.3g'
          % (T, B, worst))
    assert worst <= 1e-4
