"""Persistent generation sample loop (csrc/gen_mlp.hip) against the per-sample kernel path,
the teacher-forced Predictor and the sampler definition (Generator.__call__,
model.py:445-520).

* fp32: the persistent loop and the per-sample kernels must draw the SAME index stream from
  the same Exp(1) noise, and their per-step log-probs agree within 1e-4 (north star);
* bf16 (the production dtype) at configs[2] size (D = 1024, B = 128): every drawn index is
  exactly argmax(exp(logp) / q) of the log-probs the loop reports, and those log-probs are
  the teacher-forced fp32 Predictor's on the generated stream within a bf16 tolerance;
* shapes with a ragged last row group (B not a multiple of R).
"""
import numpy as np
import pytest
import torch

import recipe

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def build(cfg, seed, dtype):
    import model as M
    m = M.SampleRNN(cfg['frame_sizes'], cfg['n_rnn'], cfg['dim'], cfg['learn_h0'],
                    cfg['q_levels'], True, cfg['weight_norm'], cfg['cond_dim'], cfg['spk_dim'])
    m.compute_dtype = dtype
    pred = M.Predictor(m)
    pred.load_state_dict({k: torch.from_numpy(v.copy())
                          for k, v in recipe.make_weights(cfg, seed).items()})
    return m.to(DEV), pred.to(DEV)


def check_draws(lp, noise, seq, L):
    """The sampler definition, exactly: x_t = argmax(exp(logp_t) / q_t) (first index on ties)
    of the log-probs the loop reports -- with a diagnostic of any mismatch (its step, row and
    the log-space margin between the two candidates)."""
    drawn = torch.argmax(torch.exp(lp) / noise.permute(1, 0, 2), dim=-1)
    got = seq[:, L:]
    bad = (drawn != got).nonzero()
    if bad.numel():
        sc = lp.double() - torch.log(noise.permute(1, 0, 2).double())
        info = []
        for b, t in bad[:8].tolist():
            info.append('row %d step %d (mod 16: %d): drawn %d score %.7g, loop %d score %.7g'
                        % (b, t, t % 16, drawn[b, t].item(), sc[b, t, drawn[b, t]].item(),
                           got[b, t].item(), sc[b, t, got[b, t]].item()))
        raise AssertionError('%d of %d draws differ: %s' % (bad.shape[0], got.numel(),
                                                             '; '.join(info)))


def generate(m, n_seqs, cond, spk, persistent, **kw):
    import model as M
    gen = M.Generator(m, True)
    _, lp = gen(n_seqs, 0, cond, spk, return_logp=True, persistent=persistent, **kw)
    return gen.last_sequences.cpu(), lp.cpu()


@pytest.mark.parametrize('D,B,n_cond,n_rnn', [(64, 5, 3, 1), (32, 3, 2, 2), (256, 24, 2, 1),
                                              (512, 40, 2, 1), (1024, 128, 2, 1),
                                              (1024, 9, 2, 1)])
def test_persistent_matches_per_sample_fp32(hip, D, B, n_cond, n_rnn):
    cfg = dict(recipe.CONFIGS['t3'], dim=D, n_rnn=n_rnn)
    m, _ = build(cfg, 7, torch.float32)
    assert hip.gen_persistent_rows(torch.float32, B, D, 16) > 0
    cond = recipe.synth_cond((B, n_cond, cfg['cond_dim']), 4)
    spk = np.arange(B) % cfg['spk_dim']
    noise = torch.from_numpy(recipe.synth_noise((n_cond * 64, B, 256), 9))
    s1, l1 = generate(m, B, cond, spk, True, noise=noise)
    s0, l0 = generate(m, B, cond, spk, False, noise=noise)
    assert torch.equal(s1, s0)
    torch.testing.assert_close(l1, l0, atol=1e-4, rtol=0)


@pytest.mark.parametrize('B,tg', [(128, '1'), (128, '0'), (120, '1'), (9, '1')])
def test_persistent_bf16_d1024(hip, monkeypatch, B, tg):
    monkeypatch.setenv('SRNN_GEN_TICK_GEMM', tg)
    cfg = recipe.CONFIGS['big']
    m, pred = build(cfg, 11, torch.bfloat16)
    assert hip.gen_persistent_rows(torch.bfloat16, B, 1024, 16) > 0
    n_cond = 2
    cond = recipe.synth_cond((B, n_cond, cfg['cond_dim']), 5)
    spk = np.arange(B) % cfg['spk_dim']
    noise = torch.from_numpy(recipe.synth_noise((n_cond * 64, B, 256), 3))
    seq, lp = generate(m, B, cond, spk, True, noise=noise)
    L = m.lookback
    check_draws(lp, noise, seq, L)
    # teacher-forced fp32 Predictor on the generated stream: bf16 tolerance on log-probs
    m.compute_dtype = torch.float32
    with torch.no_grad():
        tf = pred(seq[:, :-1], True, torch.from_numpy(cond),
                  torch.from_numpy(spk).reshape(-1, 1)).cpu()
    err = (tf - lp).abs()
    assert err.max().item() < 0.25, err.max().item()
    assert err.mean().item() < 0.02, err.mean().item()


def test_bf16_long_run_drift_d1024(hip):
    """configs[2]'s full utterance length in bf16: 750 top-tier ticks (48,000 samples, 3 s)
    through the persistent loop, then the fp32 teacher-forced Predictor (the reference's
    precision, pinned to its goldens) re-runs the whole recurrence along the generated stream
    in TBPTT chunks with the hidden state carried.  The bf16 loop's log-probs stay within the
    bf16 tolerance of the fp32 ones over the whole run, and the error does not grow with time
    (hidden-state drift): the last tenth's mean error is within 1.5x the first tenth's."""
    import model as M
    cfg = recipe.CONFIGS['big']
    m, pred = build(cfg, 17, torch.bfloat16)
    B, n_cond = 16, 750
    cond = recipe.synth_cond((B, n_cond, cfg['cond_dim']), 8)
    spk = np.arange(B) % cfg['spk_dim']
    gen = M.Generator(m, True)
    _, lp = gen(B, 0, cond, spk, sampler='philox', seed=77, return_logp=True)
    seq = gen.last_sequences
    L = m.lookback
    T = n_cond * L
    assert lp.shape == (B, T, 256) and torch.isfinite(lp).all()
    m.compute_dtype = torch.float32
    condt = torch.from_numpy(cond)
    spkt = torch.from_numpy(spk).reshape(-1, 1)
    Tc = 75 * L                                      # 4,800 samples per TBPTT chunk
    emean, emax = [], []
    with torch.no_grad():
        for c in range(T // Tc):
            tf = pred(seq[:, c * Tc: c * Tc + L + Tc - 1], c == 0,
                      condt[:, c * Tc // L:(c + 1) * Tc // L], spkt)
            d = (tf - lp[:, c * Tc:(c + 1) * Tc]).abs()
            emean.append(d.mean(-1))                  # (B, Tc): mean over the 256 levels
            emax.append(d.amax().item())
    err = torch.cat(emean, 1)                         # (B, T)
    tenth = T // 10
    first, last = err[:, :tenth].mean().item(), err[:, -tenth:].mean().item()
    print('bf16 vs fp32 teacher-forced over %d steps: max %.4f mean %.5f first tenth %.5f '
          'last tenth %.5f' % (T, max(emax), err.mean().item(), first, last))
    assert max(emax) < 0.25, max(emax)
    assert err.mean().item() < 0.02, err.mean().item()
    assert last <= 1.5 * first + 1e-3, (first, last)


def test_config_e_bf16_d1024(hip):
    """configs[4] at full width: 4 tiers FS=[16,4,4], look-ahead conditioning (C = 86),
    D = 1024, 128 utterances (one GPU's share of 1024), bf16 persistent loop.  Same sampler
    identity and teacher-forced bound as the 3-tier test; 2 top-tier frames = 512 samples."""
    cfg = dict(recipe.CONFIGS['t4la'], dim=1024)
    m, pred = build(cfg, 13, torch.bfloat16)
    B, n_cond = 128, 2
    assert hip.gen_persistent_rows(torch.bfloat16, B, 1024, 16) > 0
    cond = recipe.synth_cond((B, n_cond, cfg['cond_dim']), 7)
    spk = np.arange(B) % cfg['spk_dim']
    L = m.lookback
    assert L == 256
    noise = torch.from_numpy(recipe.synth_noise((n_cond * L, B, 256), 4))
    seq, lp = generate(m, B, cond, spk, True, noise=noise)
    check_draws(lp, noise, seq, L)
    m.compute_dtype = torch.float32
    with torch.no_grad():
        tf = pred(seq[:, :-1], True, torch.from_numpy(cond),
                  torch.from_numpy(spk).reshape(-1, 1)).cpu()
    err = (tf - lp).abs()
    assert err.max().item() < 0.25, err.max().item()
    assert err.mean().item() < 0.02, err.mean().item()


@pytest.mark.parametrize('cfgname,D,B,persistent', [('big', 1024, 128, True),
                                                    ('t3', 256, 24, False)])
def test_folded_bottom_tick_bf16(hip, monkeypatch, cfgname, D, B, persistent):
    """bf16 folded bottom tick (gi = W_ih W_in a + G[fi], gh carried by the previous tick's
    [W_up; W_hh] GEMM) against the unfolded tick (SRNN_GEN_FOLD=0): same noise, log-probs
    within bf16 tolerance on every step whose row prefix is still identical, and the folded
    stream is the teacher-forced fp32 Predictor's within the same bound."""
    cfg = dict(recipe.CONFIGS[cfgname], dim=D)
    m, pred = build(cfg, 17, torch.bfloat16)
    n_cond = 2
    L = m.lookback
    cond = recipe.synth_cond((B, n_cond, cfg['cond_dim']), 14)
    spk = np.arange(B) % cfg['spk_dim']
    noise = torch.from_numpy(recipe.synth_noise((n_cond * L, B, 256), 15))
    monkeypatch.setenv('SRNN_GEN_FOLD', '1')
    s1, l1 = generate(m, B, cond, spk, persistent, noise=noise)
    monkeypatch.setenv('SRNN_GEN_FOLD', '0')
    s0, l0 = generate(m, B, cond, spk, persistent, noise=noise)
    # step t of row b is comparable while both streams agree on samples [L, L + t)
    same = torch.cumprod((s1[:, L:] == s0[:, L:]).int(), dim=1)
    ok = torch.cat([torch.ones(B, 1, dtype=torch.int32), same[:, :-1]], dim=1).bool()
    err = (l1 - l0).abs()[ok]             # l: (B, steps, Q), ok: (B, steps)
    assert err.max().item() < 0.25, err.max().item()
    assert err.mean().item() < 0.02, err.mean().item()
    m.compute_dtype = torch.float32
    with torch.no_grad():
        tf = pred(s1[:, :-1], True, torch.from_numpy(cond),
                  torch.from_numpy(spk).reshape(-1, 1)).cpu()
    err = (tf - l1).abs()
    assert err.max().item() < 0.25, err.max().item()
    assert err.mean().item() < 0.02, err.mean().item()


@pytest.mark.parametrize('persistent', [True, False])
def test_folded_ticks_fp32(hip, monkeypatch, persistent):
    """fp32 folded ticks (SRNN_GEN_FOLD_F32, dim % 64 == 0: gi = (W_ih W_in) a + G[fi], gh
    carried by the previous tick's [W_up; W_hh] GEMM, the folded top tick) against the
    unfolded fp32 ticks: the same index stream (the folds only reassociate fp32 sums) and
    log-probs within fp32 reassociation error."""
    cfg = dict(recipe.CONFIGS['t3'], dim=128)
    m, _ = build(cfg, 19, torch.float32)
    B, n_cond = 24, 3
    cond = recipe.synth_cond((B, n_cond, cfg['cond_dim']), 16)
    spk = np.arange(B) % cfg['spk_dim']
    noise = torch.from_numpy(recipe.synth_noise((n_cond * m.lookback, B, 256), 17))
    monkeypatch.setenv('SRNN_GEN_FOLD_F32', '1')
    s1, l1 = generate(m, B, cond, spk, persistent, noise=noise)
    monkeypatch.setenv('SRNN_GEN_FOLD_F32', '0')
    s0, l0 = generate(m, B, cond, spk, persistent, noise=noise)
    assert torch.equal(s1, s0)
    torch.testing.assert_close(l1, l0, atol=2e-5, rtol=0)


def test_persistent_philox_matches_per_sample_fp32(hip):
    """Device RNG: both paths draw Philox4x32-10(seed) noise with the same counters."""
    cfg = dict(recipe.CONFIGS['t3'], dim=128)
    m, _ = build(cfg, 3, torch.float32)
    B, n_cond = 16, 3
    cond = recipe.synth_cond((B, n_cond, cfg['cond_dim']), 6)
    spk = np.arange(B) % cfg['spk_dim']
    s1, l1 = generate(m, B, cond, spk, True, sampler='philox', seed=99)
    s0, l0 = generate(m, B, cond, spk, False, sampler='philox', seed=99)
    assert torch.equal(s1, s0)
    torch.testing.assert_close(l1, l0, atol=1e-4, rtol=0)


def test_persistent_static_map_mode(hip, monkeypatch):
    """SRNN_GEN_LOCAL=0: groups by block index with write-through (sc1) hand-offs instead of
    the XCD census; same index stream as the per-sample path."""
    monkeypatch.setenv('SRNN_GEN_LOCAL', '0')
    cfg = dict(recipe.CONFIGS['t3'], dim=256)
    m, _ = build(cfg, 5, torch.float32)
    B, n_cond = 64, 2
    cond = recipe.synth_cond((B, n_cond, cfg['cond_dim']), 8)
    spk = np.arange(B) % cfg['spk_dim']
    noise = torch.from_numpy(recipe.synth_noise((n_cond * 64, B, 256), 2))
    s1, l1 = generate(m, B, cond, spk, True, noise=noise)
    s0, l0 = generate(m, B, cond, spk, False, noise=noise)
    assert torch.equal(s1, s0)
    torch.testing.assert_close(l1, l0, atol=1e-4, rtol=0)


@pytest.mark.parametrize('sampler', ['philox', 'replay'])
def test_noise_ahead_matches_in_loop_draws(hip, monkeypatch, sampler):
    """The persistent loop's noise (log q) drawn ahead by the bottom tick's input launch is
    the noise the loop draws itself (SRNN_GEN_NOISE_AHEAD=0): identical index streams and
    log-probs, bf16 D = 1024 (the compiled-shape loop) and fp32."""
    for dtype, cfgname, B in ((torch.bfloat16, 'big', 128), (torch.float32, 't3', 24)):
        cfg = recipe.CONFIGS[cfgname]
        m, _ = build(cfg, 13, dtype)
        n_cond = 2
        cond = recipe.synth_cond((B, n_cond, cfg['cond_dim']), 12)
        spk = np.arange(B) % cfg['spk_dim']
        L = int(np.prod(cfg['frame_sizes']))
        kw = (dict(sampler='philox', seed=1234) if sampler == 'philox' else
              dict(noise=torch.from_numpy(recipe.synth_noise((n_cond * L, B, 256), 21))))
        monkeypatch.setenv('SRNN_GEN_NOISE_AHEAD', '1')
        s1, l1 = generate(m, B, cond, spk, True, **kw)
        monkeypatch.setenv('SRNN_GEN_NOISE_AHEAD', '0')
        s0, l0 = generate(m, B, cond, spk, True, **kw)
        assert torch.equal(s1, s0)
        assert torch.equal(l1, l0)


@pytest.mark.parametrize('B,n_cond', [(128, 6), (124, 2), (9, 4)])
def test_tick_gemm_in_launch_bf16(hip, monkeypatch, B, n_cond):
    """The bottom tick's [W_up; W_hh] GEMM inside the persistent launch (GenMlpArgs::tg: a
    GEMM phase, write-through stores, one grid barrier, then the sample loop) against its own
    launch (SRNN_GEN_TICK_GEMM=0): the same products in another fp32 summation order, so on
    every step whose row prefix is still identical the log-probs agree within bf16 rounding
    of the conditioning; n_cond = 6 replays the captured block twice (grid-barrier epochs
    across replays); the sampler identity and the teacher-forced fp32 bound hold."""
    cfg = recipe.CONFIGS['big']
    m, pred = build(cfg, 19, torch.bfloat16)
    L = m.lookback
    cond = recipe.synth_cond((B, n_cond, cfg['cond_dim']), 21)
    spk = np.arange(B) % cfg['spk_dim']
    noise = torch.from_numpy(recipe.synth_noise((n_cond * L, B, 256), 22))
    monkeypatch.setenv('SRNN_GEN_TICK_GEMM', '1')
    s1, l1 = generate(m, B, cond, spk, True, noise=noise)
    monkeypatch.setenv('SRNN_GEN_TICK_GEMM', '0')
    s0, l0 = generate(m, B, cond, spk, True, noise=noise)
    check_draws(l1, noise, s1, L)
    same = torch.cumprod((s1[:, L:] == s0[:, L:]).int(), dim=1)
    ok = torch.cat([torch.ones(B, 1, dtype=torch.int32), same[:, :-1]], dim=1).bool()
    err = (l1 - l0).abs()[ok]
    print('tick GEMM in launch vs own launch: %.3f of steps on identical prefixes, max %.4g '
          'mean %.3g' % (ok.float().mean().item(), err.max().item(), err.mean().item()))
    assert ok.float().mean().item() > 0.5
    assert err.max().item() < 0.1, err.max().item()
    assert err.mean().item() < 2e-3, err.mean().item()
    m.compute_dtype = torch.float32
    with torch.no_grad():
        tf = pred(s1[:, :-1], True, torch.from_numpy(cond),
                  torch.from_numpy(spk).reshape(-1, 1)).cpu()
    err = (tf - l1).abs()
    assert err.max().item() < 0.25, err.max().item()
    assert err.mean().item() < 0.02, err.mean().item()
