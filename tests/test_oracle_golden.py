"""Pin the CPU oracle (oracle/) to the reference's own outputs (tests/golden/)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest
import torch

from conftest import ROOT, golden
import recipe
import samplernn_oracle as O


@pytest.fixture(scope='module')
def culaw():
    d = os.path.join(ROOT, 'oracle')
    subprocess.check_call(['make', '-s', '-C', d])
    return ctypes.CDLL(os.path.join(d, 'build', 'libulaw_oracle.so'))


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def test_c_oracle_ulaw_kat(culaw):
    g = golden('ulaw')
    for k, fn in (('32', culaw.oracle_uquantize_f32_n), ('64', culaw.oracle_uquantize_f64_n)):
        x = np.ascontiguousarray(g['kat_x' + k])
        out = np.zeros(x.size, np.int64)
        fn(_p(x), _p(out), ctypes.c_int64(x.size), 256)
        assert np.array_equal(out, g['kat_q' + k].astype(np.int64))
    kk = np.arange(256, dtype=np.int64)
    lut = np.zeros(256, np.float32)
    culaw.oracle_udequantize_n(_p(kk), _p(lut), ctypes.c_int64(256), 256)
    assert np.array_equal(lut, g['lut'])


def test_torch_oracle_ulaw_kat():
    g = golden('ulaw')
    assert np.array_equal(O.uquantize(torch.from_numpy(g['kat_x32']), 256).numpy(), g['kat_q32'])
    assert np.array_equal(O.uquantize(torch.from_numpy(g['kat_x64']), 256).numpy(), g['kat_q64'])
    assert np.array_equal(O.udequantize(torch.arange(256), 256).numpy(), g['lut'])
    lq = np.stack([O.linear_quantize(torch.from_numpy(r), 256).numpy() for r in g['lin_x']])
    assert np.array_equal(lq, g['lin_q'])
    assert np.array_equal(O.linear_dequantize(torch.arange(256), 256).numpy(), g['lin_lut'])
    assert O.q_zero(256) == int(g['q_zero'])


def test_samples_wav_on_lut_grid():
    """samples/*.wav from the reference's checkpoint: every float32 value is a LUT entry."""
    g = golden('samples_wav')
    lut = golden('ulaw')['lut']
    assert np.all(np.isin(g['unique_values'], lut))
    f32 = [l for l, d in zip(g['lengths'], g['dtypes']) if d == 'float32']
    assert len(f32) == 17 and all(l % 80 == 0 for l in f32)


@pytest.mark.parametrize('name', ['t2', 't3', 't3r2wn', 't4la', 't3_20_4', 'big', 'e'])
def test_oracle_forward(name):
    g = golden('fwd_' + name)
    cfg = recipe.CONFIGS[name]
    m = O.from_state_dict(cfg, recipe.make_weights(cfg, int(g['weight_seed'])))
    with torch.no_grad():
        for n in range(int(g['n_chunks'])):
            lp = m.predict(torch.from_numpy(g['input_%d' % n]), bool(g['reset_%d' % n]),
                           torch.from_numpy(g['cond_%d' % n]), torch.from_numpy(g['spk_%d' % n]))
            if 'keep_rows' in g:
                np.testing.assert_allclose(lp[:, g['keep_rows']].numpy(), g['logp_rows_%d' % n],
                                           atol=2e-5, rtol=0)
            else:
                np.testing.assert_allclose(lp.numpy(), g['logp_%d' % n], atol=2e-5, rtol=0)
            for t in range(len(cfg['frame_sizes'])):
                np.testing.assert_allclose(m.hidden[t].numpy(), g['hidden_%d_tier%d' % (n, t)],
                                           atol=2e-6, rtol=0)


@pytest.mark.parametrize('name', ['t2', 't3', 't4la', 't3_20_4', 't3r2wn', 'big', 'e'])
def test_oracle_generation(name):
    g = golden('gen_' + name)
    cfg = recipe.CONFIGS[name]
    m = O.from_state_dict(cfg, recipe.make_weights(cfg, int(g['weight_seed'])))
    seq, lp = m.generate(int(g['n_seqs']), g['cond'], int(g['spk']), torch.from_numpy(g['noise']),
                         return_logp=True)
    L = m.lookback
    assert np.array_equal(seq[:, L:].numpy(), g['idx'])
    np.testing.assert_allclose(lp.numpy(), g['logp'], atol=2e-5, rtol=0)
    samples = O.udequantize(seq[:, L:], 256).numpy()
    assert np.array_equal(samples, g['samples'])


@pytest.mark.parametrize('name', ['t3', 't3r2wn', 't2'])
def test_oracle_tbptt(name):
    g = golden('tbptt_' + name)
    cfg = recipe.CONFIGS[name]
    m = O.from_state_dict(cfg, recipe.make_weights(cfg, int(g['weight_seed'])))
    names = [str(s) for s in g['names']]
    opt = O.OracleAdam([m.p[k] for k in names], lr=float(g['lr']))
    for s in range(int(g['n_steps'])):
        batch = (torch.from_numpy(g['input_%d' % s]), bool(g['reset_%d' % s]),
                 torch.from_numpy(g['target_%d' % s]), torch.from_numpy(g['cond_%d' % s]),
                 torch.from_numpy(g['spk_%d' % s]))
        loss, grads = O.tbptt_step(m, opt, names, batch)
        assert abs(loss - g['losses'][s]) < 1e-4
        if ('grad_%d/%s' % (s, names[0])) in g:
            for k, gr in zip(names, grads):
                np.testing.assert_allclose(gr.numpy(), g['grad_%d/%s' % (s, k)], atol=2e-5,
                                           rtol=1e-4, err_msg=k)
    for k in names:
        np.testing.assert_allclose(m.p[k].detach().numpy(), g['param_final/' + k], atol=1e-4,
                                   rtol=0, err_msg=k)
    for t in range(len(cfg['frame_sizes'])):
        np.testing.assert_allclose(m.hidden[t].numpy(), g['hidden_final_tier%d' % t], atol=1e-5)


@pytest.mark.parametrize('name', ['t3', 'big'])
def test_oracle_generation_from_seed(name):
    """The seed-driven default path (generate.py:200-253) on the CPU: seed -> the drop-in
    SampleRNN's init (same RNG consumption as the reference's, a13) -> bulk Exp(1) draw of the
    whole run's multinomial noise (what model.Generator's sampler='torch' does) -> the
    oracle's argmax(p / q) loop reproduces the reference's stream from that seed.  Pins the
    init RNG order and the bulk-draw == per-step-multinomial equivalence together."""
    import model as M
    g = golden('genseed_' + name)
    cfg = recipe.CONFIGS[name]
    torch.manual_seed(int(g['gen_seed']))
    M.SampleRNN(cfg['frame_sizes'], cfg['n_rnn'], cfg['dim'], cfg['learn_h0'], cfg['q_levels'],
                True, cfg['weight_norm'], cfg['cond_dim'], cfg['spk_dim'])
    n = int(g['n_seqs'])
    L = recipe.lookback(cfg)
    T = g['cond'].shape[0] * L
    noise = torch.empty(T, n, cfg['q_levels']).exponential_(1)
    m = O.from_state_dict(cfg, recipe.make_weights(cfg, int(g['weight_seed'])))
    seq = m.generate(n, g['cond'], int(g['spk']), noise)
    assert np.array_equal(seq[:, L:].numpy(), g['idx'])


@pytest.mark.parametrize('name', ['t2', 't3', 't4la', 't3_20_4', 't3r2wn', 'big', 'a'])
def test_log_space_draw_equals_ratio_draw_on_goldens(name):
    """The device sampler draws argmax_j (z_j - log q_j) (sampler.hpp), the reference
    argmax_j p_j / q_j (multinomial, model.py:514-517).  On every recorded step of every
    generation golden (reference log-probs + replayed noise) both give the reference's index:
    near-tie divergence rate 0 over these fixtures (min relative margins 2e-4 .. 5e-3)."""
    g = golden('gen_' + name)
    lp = g['logp'].astype(np.float32).transpose(1, 0, 2)         # (T, n, Q)
    q = g['noise'].astype(np.float32)
    ratio = np.argmax(np.exp(lp) / q, axis=-1).T
    logsp = np.argmax(lp - np.log(q), axis=-1).T
    assert np.array_equal(ratio, g['idx'])
    assert np.array_equal(logsp, g['idx'])


# --------------------------------------------------------------------------- round 4
# Reference-pinned fixtures at the measured dimensions (tests/golden/make_golden.py
# --only big4): configs[1]'s D = 1024 model over T = 1024 TBPTT chunks, configs[0]'s 2-tier
# D = 256 single-speaker model, and a 4,800-sample D = 1024 generation run.

@pytest.mark.parametrize('name', ['a', 'big'])
def test_oracle_tbptt_sampled(name):
    """3 TBPTT chunks through the oracle vs the reference's Trainer at T = 1024: losses,
    hidden states, gradients and final parameters within 3x the reference's own distance
    under a one-ulp weight perturbation plus the strict tolerances (conftest.within_floor)."""
    from conftest import within_floor, within_floor_sampled
    g = golden('tbptt_' + name)
    cfg = recipe.CONFIGS[name]
    m = O.from_state_dict(cfg, recipe.make_weights(cfg, int(g['weight_seed'])))
    names = [str(s) for s in g['names']]
    opt = O.OracleAdam([m.p[k] for k in names], lr=float(g['lr']))
    losses = []
    for s in range(int(g['n_steps'])):
        batch = (torch.from_numpy(g['input_%d' % s]), bool(g['reset_%d' % s]),
                 torch.from_numpy(g['target_%d' % s]), torch.from_numpy(g['cond_%d' % s]),
                 torch.from_numpy(g['spk_%d' % s]))
        loss, grads = O.tbptt_step(m, opt, names, batch)
        losses.append(loss)
        for k, gr in zip(names, grads):
            within_floor_sampled(gr.numpy(), g, 'grad_%d' % s, k, 2e-5, 1e-4)
        for t in range(len(cfg['frame_sizes'])):
            key = 'hidden_%d_tier%d' % (s, t)
            within_floor(m.hidden[t].numpy(), g[key], g, key, 2e-6)
    within_floor(losses, g['losses'], g, 'losses', 2e-5)
    for k in names:
        within_floor_sampled(m.p[k].detach().numpy(), g, 'param_final', k, 1e-4)


def test_oracle_forward_a():
    test_oracle_forward('a')


def test_oracle_generation_a():
    test_oracle_generation('a')


def test_oracle_generation_long_big():
    """4,800 samples of configs[2]'s model: the oracle's index stream equals the reference's
    (noise regenerated from the captured torch generator state), log-probs 2e-5."""
    from conftest import genlong_noise
    g = golden('genlong_big')
    cfg = recipe.CONFIGS['big']
    q = genlong_noise(g)
    m = O.from_state_dict(cfg, recipe.make_weights(cfg, int(g['weight_seed'])))
    seq, lp = m.generate(int(g['n_seqs']), g['cond'], int(g['spk']), torch.from_numpy(q),
                         return_logp=True)
    L = m.lookback
    assert np.array_equal(seq[:, L:].numpy(), g['idx'].astype(np.int64))
    np.testing.assert_allclose(lp.numpy()[:, g['logp_steps']], g['logp'], atol=2e-5, rtol=0)


def test_log_space_draw_near_tie_rate_long():
    """The log-space draw over all 9,600 steps of the long D = 1024 run equals the
    reference's argmax(p/q) draw (recorded by make_golden from the full log-probs); the
    minimum relative margin of that run is recorded in DESIGN."""
    g = golden('genlong_big')
    assert int(g['logspace_diff']) == 0
    assert float(g['margin'].min()) > 0


@pytest.mark.parametrize('name', ['a', 'big'])
def test_reference_thread_drift_within_floor(name):
    """The reference rerun at 1 thread (MKL reduction order changed, alt_* keys) stays within
    the floor the one-ulp perturbations set: they are the larger rounding-level disturbance,
    so they are the one the tolerances are built on."""
    from conftest import within_floor
    g = golden('tbptt_' + name)
    names = [str(s) for s in g['names']]
    within_floor(g['alt_losses'], g['losses'], g, 'losses', 1e-4)
    for s in range(1, int(g['n_steps'])):
        for k in names:
            key = 'grad_%d/%s' % (s, k)
            within_floor(g['smp_alt_' + key], g['smp_' + key], g, key, 1e-4, 1e-3)
    for k in names:
        key = 'param_final/' + k
        within_floor(g['smp_alt_' + key], g['smp_' + key], g, key, 2e-4)
