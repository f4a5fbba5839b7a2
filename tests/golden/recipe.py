"""Seeded, numpy-only recipes for golden weights and synthetic inputs.

Test infrastructure.  Everything here is a pure function of (config, seed) built on
numpy's PCG64, so the GPU box regenerates the exact same weights/inputs that
`make_golden.py` fed to the reference in the survey container -- no reference code
and no large weight files travel.

Parameter names and shapes follow the reference's `Predictor.state_dict()`
(model.py:18-325; nn.py:7-43):
  model.frame_level_rnns.{i}.{h0, input_expand.*, cond_expand.*, spk_embedding.*,
  spk_expand.*, rnn.{weight,bias}_{ih,hh}_l{l}, upsampling.bias,
  upsampling.conv_t.weight_{g,v}}  and  model.sample_level_mlp.{embedding, input,
  hidden, output}.*
"""
import numpy as np


def cumprod(xs):
    out, p = [], 1
    for x in xs:
        p *= int(x)
        out.append(p)
    return out


def param_shapes(frame_sizes, n_rnn, dim, q_levels, weight_norm, cond_dim, spk_dim):
    """Ordered (name, shape) list of the reference Predictor state_dict."""
    shapes = []
    nfs = cumprod(frame_sizes)
    n_tiers = len(frame_sizes)
    D = dim
    for i, (fs, n) in enumerate(zip(frame_sizes, nfs)):
        p = 'model.frame_level_rnns.%d.' % i
        is_cond = (i == n_tiers - 1)
        shapes.append((p + 'h0', (n_rnn, D)))
        if weight_norm:
            shapes.append((p + 'input_expand.weight_g', (D, 1, 1)))
            shapes.append((p + 'input_expand.weight_v', (D, n, 1)))
        else:
            shapes.append((p + 'input_expand.weight', (D, n, 1)))
        shapes.append((p + 'input_expand.bias', (D,)))
        if is_cond:
            if weight_norm:
                shapes.append((p + 'cond_expand.weight_g', (D, 1, 1)))
                shapes.append((p + 'cond_expand.weight_v', (D, cond_dim, 1)))
            else:
                shapes.append((p + 'cond_expand.weight', (D, cond_dim, 1)))
            shapes.append((p + 'cond_expand.bias', (D,)))
            shapes.append((p + 'spk_embedding.weight', (spk_dim, spk_dim)))
            if weight_norm:
                shapes.append((p + 'spk_expand.weight_g', (D, 1, 1)))
                shapes.append((p + 'spk_expand.weight_v', (D, spk_dim, 1)))
            else:
                shapes.append((p + 'spk_expand.weight', (D, spk_dim, 1)))
            shapes.append((p + 'spk_expand.bias', (D,)))
        for l in range(n_rnn):
            shapes.append((p + 'rnn.weight_ih_l%d' % l, (3 * D, D)))
            shapes.append((p + 'rnn.weight_hh_l%d' % l, (3 * D, D)))
            shapes.append((p + 'rnn.bias_ih_l%d' % l, (3 * D,)))
            shapes.append((p + 'rnn.bias_hh_l%d' % l, (3 * D,)))
        shapes.append((p + 'upsampling.bias', (D, fs)))
        # conv_t is ALWAYS weight-normed (model.py:177 tests the imported function)
        shapes.append((p + 'upsampling.conv_t.weight_g', (D, 1, 1)))
        shapes.append((p + 'upsampling.conv_t.weight_v', (D, D, fs)))
    p = 'model.sample_level_mlp.'
    Q, FS0 = q_levels, frame_sizes[0]
    shapes.append((p + 'embedding.weight', (Q, Q)))
    for name, shp, has_bias in (('input', (D, Q, FS0), False), ('hidden', (D, D, 1), True),
                                ('output', (Q, D, 1), True)):
        if weight_norm:
            shapes.append((p + name + '.weight_g', (shp[0], 1, 1)))
            shapes.append((p + name + '.weight_v', shp))
        else:
            shapes.append((p + name + '.weight', shp))
        if has_bias:
            shapes.append((p + name + '.bias', (shp[0],)))
    return shapes


def _scale(name, shape):
    """Uniform half-range giving O(1) activations and non-trivial biases."""
    if name.endswith('h0'):
        return 0.5
    if name.endswith('spk_embedding.weight') or name.endswith('embedding.weight'):
        return 1.0
    if name.endswith('weight_g'):
        return None  # handled separately (positive)
    if 'bias' in name:
        return 0.1
    # fan_in = prod(shape[1:]) except ConvTranspose (in, out, k) where fan_in = in
    if 'conv_t' in name:
        fan_in = shape[0]
    else:
        fan_in = int(np.prod(shape[1:]))
    s = np.sqrt(3.0 / fan_in)
    if 'sample_level_mlp.output' in name:
        s *= 3.0  # peaky output distribution -> realistic sampling margins
    if 'sample_level_mlp.input' in name:
        s *= 2.0
    return s


def make_weights(cfg, seed):
    """state_dict (name -> float32 ndarray) for config dict `cfg`."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = {}
    for name, shape in param_shapes(cfg['frame_sizes'], cfg['n_rnn'], cfg['dim'],
                                    cfg['q_levels'], cfg['weight_norm'], cfg['cond_dim'],
                                    cfg['spk_dim']):
        if name.endswith('weight_g'):
            a = rng.uniform(0.5, 1.5, size=shape)
        else:
            s = _scale(name, shape)
            a = rng.uniform(-s, s, size=shape)
        out[name] = a.astype(np.float32)
    return out


def lookback(cfg):
    return cumprod(cfg['frame_sizes'])[-1]


def synth_audio(n, seed):
    """Sum of three sinusoids + Laplacian noise, peak 0.9, float64."""
    rng = np.random.Generator(np.random.PCG64(seed))
    t = np.arange(n, dtype=np.float64) / 16000.0
    x = np.zeros(n)
    for _ in range(3):
        f = rng.uniform(80.0, 2000.0)
        ph = rng.uniform(0, 2 * np.pi)
        a = rng.uniform(0.1, 0.4)
        x += a * np.sin(2 * np.pi * f * t + ph)
    x += rng.laplace(0.0, 0.05, size=n)
    x *= 0.9 / np.max(np.abs(x))
    return x


def synth_cond(shape, seed):
    """Min-max-normalised-looking conditioners U[0,1), float64 (dataset.py dtype)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.uniform(0.0, 1.0, size=shape)


def synth_noise(shape, seed):
    """Exp(1) sampling noise q (argmax(p/q) sampling), float32."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.exponential(1.0, size=shape).astype(np.float32)


CONFIGS = {
    # name: model config
    't2': dict(frame_sizes=[16], n_rnn=1, dim=32, q_levels=256, weight_norm=False,
               cond_dim=43, spk_dim=6, learn_h0=True),
    't3': dict(frame_sizes=[16, 4], n_rnn=1, dim=48, q_levels=256, weight_norm=False,
               cond_dim=43, spk_dim=6, learn_h0=True),
    't3r2wn': dict(frame_sizes=[16, 4], n_rnn=2, dim=32, q_levels=256, weight_norm=True,
                   cond_dim=43, spk_dim=6, learn_h0=True),
    't4la': dict(frame_sizes=[16, 4, 4], n_rnn=1, dim=32, q_levels=256, weight_norm=False,
                 cond_dim=86, spk_dim=6, learn_h0=True),
    't3_20_4': dict(frame_sizes=[20, 4], n_rnn=2, dim=32, q_levels=256, weight_norm=False,
                    cond_dim=43, spk_dim=6, learn_h0=False),
    'big': dict(frame_sizes=[16, 4], n_rnn=1, dim=1024, q_levels=256, weight_norm=False,
                cond_dim=43, spk_dim=6, learn_h0=True),
    # configs[4]: 4-tier, dim 1024, FS [16, 4, 4], look-ahead conditioning (train.py:213:
    # cond_dim x (1 + look_ahead) = 86), 6 speakers
    'e': dict(frame_sizes=[16, 4, 4], n_rnn=1, dim=1024, q_levels=256, weight_norm=False,
              cond_dim=86, spk_dim=6, learn_h0=True),
    # configs[0]: 2-tier, dim 256, one speaker (train.py:201 counts speaker directories, so a
    # single-speaker dataset gives spk_dim = 1), the train.py defaults otherwise
    'a': dict(frame_sizes=[16], n_rnn=1, dim=256, q_levels=256, weight_norm=False,
              cond_dim=43, spk_dim=1, learn_h0=True),
}


def sample_index(numel, name, k=4096):
    """Fixed seeded subset of flat entries of a tensor (the large fixtures store these
    entries, a sum and an L2 norm per tensor instead of the full tensor)."""
    if numel <= k:
        return np.arange(numel)
    h = sum((i + 1) * ord(c) for i, c in enumerate(name)) & 0xFFFFFFFF
    rng = np.random.Generator(np.random.PCG64(h))
    return np.sort(rng.choice(numel, size=k, replace=False))
