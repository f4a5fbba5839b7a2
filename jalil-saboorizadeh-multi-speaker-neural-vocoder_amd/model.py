"""Drop-in for the reference's model.py (model.py:1-520), MI355X-native.

Same classes, constructor signatures, attributes, state_dict keys and init recipe
(RNG consumption order) as the reference -- SampleRNN, FrameLevelRNN, SampleLevelMLP,
Runner, Predictor, Generator -- so train.py / generate.py bind unchanged.  Every
forward/backward runs on the hand-written HIP kernels of libsamplernn_hip.so:

  * FrameLevelRNN  -> srnn::tier_fwd / tier_bwd (custom_ops.py; tier_forward /
    tier_backward here): input / cond / speaker projections (MFMA GEMMs with fused bias +
    upper-tier add), the GRU input projection for all frames in one GEMM, the recurrence as
    one persistent sweep per layer (gru_xcd.hip) or per-step kernels, LearnedUpsampling1d as
    one GEMM; the backward mirrors it.
  * SampleLevelMLP -> srnn::mlp_fwd / mlp_bwd (mlp_forward / mlp_backward): embedding . conv
    folded into a per-tap table, L1 as a gather-sum, hidden / output GEMMs with fused bias /
    ReLU, log-softmax kernel; with sequence_nll_loss_bits the loss backward is fused in.
  * Generator      -> srnn::generate: the whole autoregressive loop on the device (persistent
    sample loop + tier ticks, captured as a hipGraph; no per-sample host round trip).

Numerics: fp32 by default (parity mode, logits within 1e-4 of the reference);
`SampleRNN.compute_dtype = torch.bfloat16` (or env SRNN_COMPUTE_DTYPE=bf16) runs the
matmuls on bf16 MFMA with fp32 accumulation, fp32 master weights and fp32 recurrences.
"""
import ctypes
import os

import numpy as np
import torch
from torch.nn import init

import custom_ops
import nn
import utils
import samplernn_hip as H

verbose = False
# (tests) how often a fused side result was consumed, and which recurrence kernels ran
_STATS = {'fused_colsum': 0, 'fused_lp': 0, 'csum_epi': 0, 'lsm_epi': 0, 'gru_xcd_fwd': 0, 'gru_xcd_bwd': 0, 'gru_seq': 0,
          'gru_cell_steps': 0, 'gru_cell_bwd_steps': 0}


def _default_dtype():
    v = os.environ.get('SRNN_COMPUTE_DTYPE', 'fp32').lower()
    return torch.bfloat16 if v in ('bf16', 'bfloat16') else torch.float32


class _GRUParams(torch.nn.Module):
    """Parameter container with torch.nn.GRU's names and reset_parameters RNG order
    (weight_ih_l{l}, weight_hh_l{l}, bias_ih_l{l}, bias_hh_l{l}); the recurrence itself
    runs in the HIP gru_cell kernel."""

    def __init__(self, input_size, hidden_size, num_layers):
        super().__init__()
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        for l in range(num_layers):
            isz = input_size if l == 0 else hidden_size
            self.register_parameter('weight_ih_l%d' % l,
                                    torch.nn.Parameter(torch.empty(3 * hidden_size, isz)))
            self.register_parameter('weight_hh_l%d' % l,
                                    torch.nn.Parameter(torch.empty(3 * hidden_size, hidden_size)))
            self.register_parameter('bias_ih_l%d' % l,
                                    torch.nn.Parameter(torch.empty(3 * hidden_size)))
            self.register_parameter('bias_hh_l%d' % l,
                                    torch.nn.Parameter(torch.empty(3 * hidden_size)))
        stdv = 1.0 / np.sqrt(hidden_size)
        for p in self.parameters():
            init.uniform_(p, -stdv, stdv)


class SampleRNN(torch.nn.Module):
    """model.py:18-62."""

    def __init__(self, frame_sizes, n_rnn, dim, learn_h0, q_levels, ulaw, weight_norm, cond_dim,
                 spk_dim, qrnn=False):
        super().__init__()
        self.dim = dim
        self.q_levels = q_levels
        self.ulaw = ulaw
        self.cond_dim = cond_dim
        self.spk_dim = spk_dim
        self.frame_sizes = [int(f) for f in frame_sizes]
        self.n_rnn = n_rnn
        self.compute_dtype = _default_dtype()
        self.dequantize = utils.udequantize if ulaw else utils.linear_dequantize
        ns_frame_samples = list(map(int, np.cumprod(frame_sizes)))
        is_cond = [False] * len(frame_sizes)
        is_cond[-1] = True
        self.frame_level_rnns = torch.nn.ModuleList([
            FrameLevelRNN(frame_size, n_frame_samples, n_rnn, dim, learn_h0, c, cond_dim,
                          spk_dim, weight_norm, qrnn)
            for (frame_size, n_frame_samples, c) in zip(frame_sizes, ns_frame_samples, is_cond)
        ])
        self.sample_level_mlp = SampleLevelMLP(frame_sizes[0], dim, q_levels, weight_norm)
        self.frame_level_rnns[0].__dict__['_feeds_mlp'] = True
        for m in self.modules():
            if m is not self:
                m.__dict__['_root'] = self

    @property
    def lookback(self):
        return self.frame_level_rnns[-1].n_frame_samples


class FrameLevelRNN(torch.nn.Module):
    """model.py:65-263 (parameters, init recipe, forward contract)."""

    def __init__(self, frame_size, n_frame_samples, n_rnn, dim, learn_h0, is_cond, cond_dim,
                 spk_dim, w_norm, qrnn):
        super().__init__()
        self.frame_size = frame_size
        self.n_frame_samples = n_frame_samples
        self.dim = dim
        self.cond_dim = cond_dim
        self.spk_dim = spk_dim
        self.weight_norm = w_norm
        self.qrnn = qrnn
        self.n_rnn = n_rnn
        self.is_cond = is_cond
        h0 = torch.zeros(n_rnn, dim)
        if learn_h0:
            self.h0 = torch.nn.Parameter(h0)
        else:
            self.register_buffer('h0', h0)
        self.input_expand = torch.nn.Conv1d(n_frame_samples, dim, kernel_size=1)
        if is_cond:
            self.cond_expand = torch.nn.Conv1d(cond_dim, dim, kernel_size=1)
            init.kaiming_uniform_(self.cond_expand.weight)
            init.constant_(self.cond_expand.bias, 0)
            self.spk_embedding = torch.nn.Embedding(spk_dim, spk_dim)
            self.spk_expand = torch.nn.Conv1d(spk_dim, dim, kernel_size=1)
            init.kaiming_uniform_(self.spk_expand.weight)
            init.constant_(self.spk_expand.bias, 0)
            if w_norm:
                nn.apply_weight_norm(self.cond_expand)
                nn.apply_weight_norm(self.spk_expand)
        else:
            self.cond_expand = None
            self.spk_expand = None
            self.spk_embedding = None
        init.kaiming_uniform_(self.input_expand.weight)
        init.constant_(self.input_expand.bias, 0)
        if w_norm:
            nn.apply_weight_norm(self.input_expand)
        # qrnn=True in the reference also builds a torch GRU (model.py:133-139)
        self.rnn = _GRUParams(dim, dim, n_rnn)
        for i in range(n_rnn):
            nn.concat_init(getattr(self.rnn, 'weight_ih_l%d' % i),
                           [nn.lecun_uniform, nn.lecun_uniform, nn.lecun_uniform])
            init.constant_(getattr(self.rnn, 'bias_ih_l%d' % i), 0)
            nn.concat_init(getattr(self.rnn, 'weight_hh_l%d' % i),
                           [nn.lecun_uniform, nn.lecun_uniform, init.orthogonal_])
            init.constant_(getattr(self.rnn, 'bias_hh_l%d' % i), 0)
        self.upsampling = nn.LearnedUpsampling1d(dim, dim, frame_size)
        init.uniform_(self.upsampling.conv_t.weight, -np.sqrt(6 / dim), np.sqrt(6 / dim))
        init.constant_(self.upsampling.bias, 0)
        # always weight-normed: model.py:177 tests the imported function, not the flag
        nn.apply_weight_norm(self.upsampling.conv_t)

    # parameter tensors in the order tier_forward consumes them (srnn::tier_fwd's params)
    def _param_list(self):
        ps = []
        ps += nn.weight_params(self.input_expand) + [self.input_expand.bias]
        if self.is_cond:
            ps += nn.weight_params(self.cond_expand) + [self.cond_expand.bias]
            ps += [self.spk_embedding.weight]
            ps += nn.weight_params(self.spk_expand) + [self.spk_expand.bias]
        for l in range(self.n_rnn):
            ps += [getattr(self.rnn, 'weight_ih_l%d' % l), getattr(self.rnn, 'weight_hh_l%d' % l),
                   getattr(self.rnn, 'bias_ih_l%d' % l), getattr(self.rnn, 'bias_hh_l%d' % l)]
        ps += nn.weight_params(self.upsampling.conv_t) + [self.upsampling.bias]
        return ps

    def forward(self, prev_samples, upper_tier_conditioning, hidden, cond, spk, writer,
                iterations):
        """model.py:180-263: (B,F,nfs) samples -> ((B, F*frame_size, D) conditioning, hidden)."""
        H.need_cuda(prev_samples)
        dev = prev_samples.device
        if cond is not None:
            cond = cond.to(dev)
        if spk is not None:
            spk = spk.to(dev).long()
        h0 = self.h0
        ps = self._param_list()
        # the registered op srnn::tier_fwd (custom_ops.py; autograd: srnn::tier_bwd)
        out, h = custom_ops.tier(prev_samples.float().contiguous(),
                                 None if upper_tier_conditioning is None
                                 else upper_tier_conditioning.contiguous(),
                                 cond, spk, None if hidden is None else hidden.contiguous(),
                                 h0, ps, tier_meta(self))
        return out, h


def _wcast(mod, T):
    """Effective weight of a conv module in the compute dtype: the cached copy of the plain
    parameter (samplernn_hip.cast_param), or a cast of the weight-normed weight."""
    if hasattr(mod, 'weight_g'):
        return H.cast(nn.weight_of(mod), T)
    return H.cast_param(mod.weight, T)


def _wcast_t(mod, T):
    """Transposed effective weight (in, out) of a k = 1 conv in the compute dtype, permuted
    straight from the fp32 weight (one launch; weight norm applied first)."""
    w = nn.weight_of(mod)
    o, i = w.shape[0], w.shape[1]
    return H.permute3(w.reshape(1, o, i), (0, 2, 1), dtype=T).reshape(i, o)


def _dt(mod):
    T = mod.__dict__.get('T')
    if T is not None:
        return T
    root = mod.__dict__.get('_root')
    return root.compute_dtype if root is not None else torch.float32


class _Conv:
    """A conv's parameters as the weight helpers of nn.py see them: `weight`, or
    `weight_g` / `weight_v` under weight norm."""

    def __init__(self, ts):
        if len(ts) == 2:
            self.weight_g, self.weight_v = ts
        else:
            self.weight = ts[0]


class TierSpec:
    """Static description of one FrameLevelRNN for the srnn::tier_* ops: the meta ints
    (tier_meta) plus the parameter list in FrameLevelRNN._param_list order."""

    def __init__(self, meta, ps):
        (self.dim, self.n_frame_samples, self.frame_size, self.n_rnn, is_cond, feeds, dt,
         wn_ie, wn_c, wn_s, wn_up) = [int(v) for v in meta[:11]]
        self.is_cond = bool(is_cond)
        self.T = torch.bfloat16 if dt else torch.float32
        self._feeds_mlp = bool(feeds)
        it = iter(ps)

        def take(wn):
            return _Conv([next(it) for _ in range(2 if wn else 1)])
        self.input_expand = take(wn_ie)
        next(it)
        if self.is_cond:
            self.cond_expand = take(wn_c)
            next(it)
            next(it)
            self.spk_expand = take(wn_s)
            next(it)
        for _ in range(4 * self.n_rnn):
            next(it)
        self.upsampling = _State()
        self.upsampling.conv_t = take(wn_up)


def tier_meta(mod):
    """The meta ints of TierSpec for a FrameLevelRNN."""
    wn = lambda m: int(hasattr(m, 'weight_g'))  # noqa: E731
    return [mod.dim, mod.n_frame_samples, mod.frame_size, mod.n_rnn, int(mod.is_cond),
            int(bool(mod.__dict__.get('_feeds_mlp'))), H.dcode(_dt(mod)),
            wn(mod.input_expand), wn(mod.cond_expand) if mod.is_cond else 0,
            wn(mod.spk_expand) if mod.is_cond else 0, wn(mod.upsampling.conv_t)]


class MlpSpec:
    """Static description of the SampleLevelMLP for the srnn::mlp_* ops (mlp_meta + the
    parameter list in SampleLevelMLP._param_list order)."""

    def __init__(self, meta, ps):
        self.q_levels, self.dim, self.frame_size, dt, wn = [int(v) for v in meta[:5]]
        self.T = torch.bfloat16 if dt else torch.float32
        it = iter(ps)

        def take():
            return _Conv([next(it) for _ in range(2 if wn else 1)])
        self.embedding = _Conv([next(it)])
        self.input = take()
        self.hidden = take()
        self.hidden.bias = next(it)
        self.output = take()
        self.output.bias = next(it)


def mlp_meta(mlp):
    return [mlp.q_levels, mlp.dim, mlp.frame_size, H.dcode(_dt(mlp)),
            int(hasattr(mlp.hidden, 'weight_g'))]


class _State:
    """What a tier / MLP forward keeps for its backward (custom_ops stash)."""


def tier_forward(mod, prev, upper, cond, spk, hidden, h0, ps):
    """FrameLevelRNN forward (model.py:180-263) on the HIP kernels: returns (Y, h_new, state)
    with state what tier_backward needs (srnn::tier_fwd, custom_ops.py)."""
    T = _dt(mod)
    B, Fr, nfs = prev.shape
    D = mod.dim
    L = mod.n_rnn
    dev = prev.device
    it = iter(ps)

    def take_w(m):
        return [next(it) for _ in nn.weight_params(m)]

    ie_p = take_w(mod.input_expand)
    ie_b = next(it)
    W_ie = _wcast(mod.input_expand, T).reshape(D, nfs)
    prevT = H.cast(prev.reshape(B * Fr, nfs), T)
    lp = T != torch.float32
    # In the low-precision mode only the compute-dtype copy of the first GRU layer's input
    # is ever read, so the last projection writes it directly (no fp32 x0, no cast); the
    # fp32 (parity) mode keeps the reference's summation order.
    x0 = H.linear(prevT, W_ie, bias=ie_b,
                  cin=None if upper is None else upper.reshape(B * Fr, D),
                  beta=0.0 if upper is None else 1.0,
                  out_dtype=T if lp and not mod.is_cond else torch.float32)
    condT = spk_embT = W_c = W_s = None
    if mod.is_cond:
        take_w(mod.cond_expand)
        c_b = next(it)
        E_s = next(it)
        take_w(mod.spk_expand)
        s_b = next(it)
        C = cond.shape[-1]
        W_c = _wcast(mod.cond_expand, T).reshape(D, C)
        condT = H.cast(cond.reshape(B * Fr, C).float().contiguous(), T)
        S = E_s.shape[1]
        spk_flat = spk.reshape(B).contiguous()
        spk_emb = torch.empty((B, S), device=dev, dtype=torch.float32)
        H.lib().call('srnn_gather_rows', H.ptr(E_s), S, H.ptr(spk_flat), B, S, H.ptr(spk_emb),
                     H.F32, S, H.stream())
        spk_embT = H.cast(spk_emb, T)
        W_s = _wcast(mod.spk_expand, T).reshape(D, S)
        spk_proj = H.linear(spk_embT, W_s, bias=s_b)
        if lp:
            H.lib().call('srnn_add_bcast_rows', H.ptr(x0), H.ptr(spk_proj), B, Fr, D, D,
                         H.stream())
            x0 = H.linear(condT, W_c, bias=c_b, cin=x0, beta=1.0, out_dtype=T)
        else:
            H.linear(condT, W_c, bias=c_b, cin=x0, beta=1.0, out=x0)
            H.lib().call('srnn_add_bcast_rows', H.ptr(x0), H.ptr(spk_proj), B, Fr, D, D,
                         H.stream())
    else:
        spk_flat = None
    reset = hidden is None
    if reset:   # model.py:224-228
        h_in = h0.detach().reshape(L, 1, D).expand(L, B, D).contiguous()
    else:
        h_in = hidden.float().contiguous()
    Wih, Whh, WhhF, bih, bhh = [], [], [], [], []
    xs, outs, outsT, gates, hprevs = [], [], [], [], []
    X = x0
    for l in range(L):
        wih, whh, b_ih, b_hh = next(it), next(it), next(it), next(it)
        Wih.append(H.cast_param(wih, T))
        Whh.append(H.cast_param(whh, T))
        WhhF.append(whh)
        bih.append(b_ih)
        bhh.append(b_hh)
        XT = H.cast(X, T)
        gi = H.linear(XT, Wih[l], bias=b_ih)                      # (B*F, 3D)
        out = torch.empty((B, Fr, D), device=dev, dtype=torch.float32)
        outT = torch.empty((B, Fr, D), device=dev, dtype=T) if lp else out
        gt = torch.empty((B, Fr, 4 * D), device=dev, dtype=torch.float32)
        hpf = h_in[l]
        xw = H.gru_xcd_work_bytes(T, B, D) if lp else 0
        # (the XCD sweep reads the fp32 state itself; the other paths take a T copy)
        hpT = H.cast(hpf, T) if xw == 0 else None
        seq = lp and (xw > 0 or H.gru_seq_supported(T, B, D))
        if seq:
            H.before_persistent_sweep()
        hprevT = None
        if xw > 0:
            # whole sequence in one persistent launch, row groups per XCD, W_hh in VGPRs;
            # it also writes the previous-state sequence [h0, h_0 .. h_{F-2}] in bf16 for
            # the backward's W_hh gradient
            work = torch.empty(xw, device=dev, dtype=torch.uint8)
            hprevT = torch.empty((B, Fr, D), device=dev, dtype=T)
            _STATS['gru_xcd_fwd'] += 1
            ev = H.roof_begin()
            H.lib().call('srnn_gru_xcd_fwd2', H.dcode(T), B, D, Fr, H.ptr(gi), Fr * 3 * D,
                         3 * D, H.ptr(hpf), H.ptr(Whh[l]), H.ptr(b_hh), H.ptr(out),
                         H.ptr(outT), Fr * D, D, H.ptr(gt), Fr * 4 * D, 4 * D,
                         H.ptr(hprevT), H.ptr(work), xw, H.stream())
            H.roof_end('gru_xcd_fwd', ev, 2.0 * B * Fr * 3 * D * D)
        elif seq:
            # whole sequence in one persistent launch (W_hh resident in LDS)
            work = torch.empty(64 * ((B + 31) // 32) + 1, device=dev, dtype=torch.int32)
            _STATS['gru_seq'] += 1
            H.lib().call('srnn_gru_seq_fwd', H.dcode(T), B, D, Fr, H.ptr(gi), Fr * 3 * D,
                         3 * D, H.ptr(hpf), H.ptr(hpT), H.ptr(Whh[l]), H.ptr(b_hh),
                         H.ptr(out), H.ptr(outT), Fr * D, D, H.ptr(gt), Fr * 4 * D, 4 * D,
                         H.ptr(work), work.numel() * 4, H.stream())
        _STATS['gru_cell_steps'] += 0 if seq else Fr
        for t in range(0 if not seq else Fr, Fr):
            if t == 0:
                hp_t, hp_f, ldh = hpT, hpf, D
            else:
                hp_t, hp_f, ldh = outT[:, t - 1], out[:, t - 1], Fr * D
            H.lib().call('srnn_gru_cell', H.dcode(T), B, D, D, None, 0, None, None,
                         H.ptr(gi[t:]), Fr * 3 * D, H.ptr(hp_t), ldh, H.ptr(hp_f), ldh,
                         H.ptr(Whh[l]), H.ptr(b_hh), H.ptr(out[:, t]), Fr * D,
                         H.ptr(outT[:, t]) if lp else None, Fr * D, H.ptr(gt[:, t]),
                         Fr * 4 * D, H.stream())
        xs.append(XT)
        hprevs.append(hprevT)
        outs.append(out)
        outsT.append(outT)
        gates.append(gt)
        X = out.reshape(B * Fr, D)
    up_p = take_w(mod.upsampling.conv_t)
    up_b = next(it)
    k = mod.frame_size
    W_up = nn.convt_operand(mod.upsampling.conv_t, T)                        # (k, D, D)
    b_up = H.permute3(up_b.reshape(1, D, k), (0, 2, 1)).reshape(k * D)
    # the bottom tier feeds the MLP's gather directly: its upsampled output (and so the
    # gradient coming back) is in the compute dtype; upper tiers stay fp32 (Cin input)
    y_dt = T if mod.__dict__.get('_feeds_mlp') else torch.float32
    Y = H.linear(outsT[-1].reshape(B * Fr, D), W_up.reshape(k * D, D), bias=b_up,
                 out_dtype=y_dt)
    h_new = torch.stack([o[:, -1] for o in outs], 0)
    ctx = _State()
    ctx.mod = mod
    ctx.reset = reset
    ctx.has_upper = upper is not None
    ctx.dims = (B, Fr, nfs, D, L, k)
    ctx.T = T
    ctx.saved_tensors = (prevT, condT, spk_embT, spk_flat, h_in, W_ie, W_c, W_s, W_up,
                         *Wih, *Whh, *xs, *outs, *outsT, *gates, *WhhF, *hprevs)
    return Y.reshape(B, Fr * k, D), h_new, ctx


def tier_backward(ctx, dY, need_h0):
    """Backward of tier_forward: (d_upper or None, dh0 or None, [parameter gradients in
    _param_list order])."""
    mod = ctx.mod
    B, Fr, nfs, D, L, k = ctx.dims
    T = ctx.T
    lp = T != torch.float32
    sv = ctx.saved_tensors
    prevT, condT, spk_embT, spk_flat, h_in, W_ie, W_c, W_s, W_up = sv[:9]
    r = sv[9:]
    Wih, Whh = r[:L], r[L:2 * L]
    xs, outs, outsT, gates = r[2 * L:3 * L], r[3 * L:4 * L], r[4 * L:5 * L], r[5 * L:6 * L]
    WhhF = r[6 * L:7 * L]                     # the fp32 parameters W_hh
    hprevs = r[7 * L:8 * L]                   # [h_in, out[:, :F-1]] in T, or None
    dev = dY.device
    st = H.stream
    M = B * Fr
    # --- upsampling (nn.py:33-43)
    if dY.dtype == T:
        dY2 = dYT = dY.reshape(M, k * D).contiguous()
    else:
        dY2 = dY.reshape(M, k * D).float().contiguous()
        # the tier below already cast this gradient (its dx0) to the compute dtype
        lpc = getattr(dY, '_srnn_lp', None)
        if lpc is not None and lpc[1] == dY._version and lpc[0].dtype == T and \
                lpc[0].numel() == dY2.numel() and dY2.data_ptr() == dY.data_ptr():
            dYT = lpc[0].reshape(M, k * D)
            _STATS['fused_lp'] += 1
        else:
            dYT = H.cast(dY2, T)
    # weight gradient transposed, [i][j*D + o]: one row per input channel for the
    # per-channel weight-norm backward (no permute of the 16 x D x D gradient)
    dWupT = H.gemm(outsT[-1].reshape(M, D), dYT, transA=True)         # (D, k*D)
    # bias gradient: summed by the MLP's dTab pass when dY is its untouched d(upper)
    cs = getattr(dY, '_srnn_colsum', None)
    if cs is not None and cs[1] == dY._version and cs[2] == k and cs[0].numel() == k * D:
        db_up = cs[0]
        _STATS['fused_colsum'] += 1
    else:
        db_up = H.colsum(dY2, M, k * D)
    dX = H.gemm(dYT, W_up.reshape(k * D, D))                          # (M, D)
    g_up = nn.convt_grad_to_params(mod.upsampling.conv_t, dWupT)
    g_up_b = H.permute3(db_up.reshape(1, k, D), (0, 2, 1)).reshape(D, k)
    # --- GRU layers, top layer first
    g_rnn = [None] * L
    dh_in = [None] * L
    for l in reversed(range(L)):
        dOut = dX.reshape(B, Fr, D)
        # W_hh^T (D, 3D): k-contiguous operand for the deep-ring backward kernel, straight
        # from the fp32 parameter (the same bf16 values as the forward's copy, no cast pass)
        WhhT = H.permute3(WhhF[l].detach().reshape(1, 3 * D, D), (0, 2, 1), dtype=T)
        xbw = H.gru_xcd_bwd_work_bytes(T, B, D) if lp else 0
        seq = lp and (xbw > 0 or H.gru_seq_supported(T, B, D))
        ddir = [torch.empty((B, D), device=dev, dtype=torch.float32) for _ in range(2)]
        dGIT = bsum = None
        if xbw > 0:
            # the sweep writes bf16 dgh / dgi (the GEMM operands) and per-row bias sums;
            # no fp32 copies of either
            dGH = dGI = None
            dGHT = torch.empty((B, Fr, 3 * D), device=dev, dtype=T)
            dGIT = torch.empty((B, Fr, 3 * D), device=dev, dtype=T)
            bsum = torch.empty((B, 4 * D), device=dev, dtype=torch.float32)
        else:
            dGH = torch.empty((B, Fr, 3 * D), device=dev, dtype=torch.float32)
            dGHT = torch.empty((B, Fr, 3 * D), device=dev, dtype=T) if lp else dGH
            dGI = torch.empty((B, Fr, 3 * D), device=dev, dtype=torch.float32)
        if seq:
            H.before_persistent_sweep()   # (DP: in-flight all-reduces finish first)
        if xbw > 0:
            # reverse sweep in one persistent launch, row groups per XCD, W_hh^T in VGPRs
            work = torch.empty(xbw, device=dev, dtype=torch.uint8)
            dOutc = dOut.contiguous()
            _STATS['gru_xcd_bwd'] += 1
            ev = H.roof_begin()
            H.lib().call('srnn_gru_xcd_bwd2', H.dcode(T), B, D, Fr, H.ptr(dOutc), Fr * D, D,
                         H.ptr(gates[l]), Fr * 4 * D, 4 * D, H.ptr(outs[l]), Fr * D, D,
                         H.ptr(h_in[l]), H.ptr(WhhT), None, H.ptr(dGHT), None, H.ptr(dGIT),
                         H.ptr(bsum), Fr * 3 * D, 3 * D, H.ptr(ddir[0]), H.ptr(work), xbw,
                         st())
            # (the dgh_{t+1} W_hh products of steps 1 .. F-1; step F-1 has none)
            H.roof_end('gru_xcd_bwd', ev, 2.0 * B * (Fr - 1) * 3 * D * D)
        elif seq:
            # the whole reverse sweep in one persistent launch (W_hh^T resident in LDS)
            work = torch.empty(64 * ((B + 31) // 32) + 1, device=dev, dtype=torch.int32)
            dOutc = dOut.contiguous()
            H.lib().call('srnn_gru_seq_bwd', H.dcode(T), B, D, Fr, H.ptr(dOutc), Fr * D, D,
                         H.ptr(gates[l]), Fr * 4 * D, 4 * D, H.ptr(outs[l]), Fr * D, D,
                         H.ptr(h_in[l]), H.ptr(WhhT), H.ptr(dGH), H.ptr(dGHT), H.ptr(dGI),
                         Fr * 3 * D, 3 * D, H.ptr(ddir[0]), H.ptr(work), work.numel() * 4,
                         st())
        if seq:
            H.after_persistent_sweep()    # (DP: gradient buckets ready before it go out now)
        _STATS['gru_cell_bwd_steps'] += 0 if seq else Fr
        for t in reversed(range(Fr)) if not seq else ():
            nxt = t + 1 < Fr
            if t > 0:
                hp, ldhp = outs[l][:, t - 1], Fr * D
            else:
                hp, ldhp = h_in[l], D
            H.lib().call('srnn_gru_cell_bwd', H.dcode(T), B, D, H.ptr(dOut[:, t]), Fr * D,
                         H.ptr(dGHT[:, t + 1]) if nxt else None, Fr * 3 * D,
                         H.ptr(ddir[(t + 1) % 2]) if nxt else None, H.ptr(Whh[l]),
                         H.ptr(WhhT), H.ptr(gates[l][:, t]), Fr * 4 * D, H.ptr(hp), ldhp,
                         H.ptr(dGH[:, t]), Fr * 3 * D,
                         H.ptr(dGHT[:, t]) if lp else None, Fr * 3 * D,
                         H.ptr(dGI[:, t]), Fr * 3 * D, H.ptr(ddir[t % 2]), st())
        # dh_0 = dgh_0 . W_hh + dh_direct, as an NT product on W_hh^T (skinny ring path)
        dh_in[l] = H.gemm(dGHT[:, 0], WhhT, transB=True, M=B, N=D, K=3 * D,
                          lda=Fr * 3 * D, ldb=3 * D, cin=ddir[0], beta=1.0)
        # previous hidden states of every step: [h_in, out[:, :F-1]] (written by the
        # persistent forward sweep when it ran, else built here)
        hprevT = hprevs[l]
        if hprevT is None:
            hprevT = torch.empty((B, Fr, D), device=dev, dtype=T)
            H.lib().call('srnn_copy2d', H.F32, H.dcode(T), B, D, H.ptr(h_in[l]), D,
                         H.ptr(hprevT), Fr * D, st())
            if Fr > 1:
                H.lib().call('srnn_copy2d', H.dcode(T), H.dcode(T), B, (Fr - 1) * D,
                             H.ptr(outsT[l]), Fr * D, H.ptr(hprevT[:, 1:]), Fr * D, st())
        dW_hh = H.gemm(dGHT.reshape(M, 3 * D), hprevT.reshape(M, D), transA=True)
        if bsum is not None:
            bs = H.colsum(bsum, B, 4 * D)               # sums of [dar | daz | dghn | dan]
            db_hh = bs[:3 * D]
            db_ih = torch.cat([bs[:2 * D], bs[3 * D:]])
            dGIT = dGIT.reshape(M, 3 * D)
        else:
            dGH2, dGI2 = dGH.reshape(M, 3 * D), dGI.reshape(M, 3 * D)
            db_hh = H.colsum(dGH2, M, 3 * D)
            dGIT = H.cast(dGI2, T)
            db_ih = H.colsum(dGI2, M, 3 * D)
        dW_ih = H.gemm(dGIT, xs[l], transA=True)
        dX = H.gemm(dGIT, Wih[l])                                     # (M, D)
        g_rnn[l] = [dW_ih, dW_hh, db_ih, db_hh]
    # --- input projections
    dx0 = dX
    dx0T = H.cast(dx0, T)
    dW_ie = H.gemm(dx0T, prevT, transA=True)                         # (D, nfs)
    g_ie = nn.weight_grad_to_params(mod.input_expand, dW_ie.reshape(D, nfs, 1))
    g_ie_b = H.colsum(dx0, M, D)
    d_upper = dx0.reshape(B, Fr, D) if ctx.has_upper else None
    if d_upper is not None and dx0T is not dx0:
        d_upper._srnn_lp = (dx0T, d_upper._version)     # (the upper tier's dY cast)
    grads = g_ie + [g_ie_b]
    if mod.is_cond:
        C = condT.shape[1]
        S = spk_embT.shape[1]
        dW_c = H.gemm(dx0T, condT, transA=True)                      # (D, C)
        grads += nn.weight_grad_to_params(mod.cond_expand, dW_c.reshape(D, C, 1))
        grads += [g_ie_b.clone()]                                    # cond bias grad
        dspk = torch.empty((B, D), device=dev, dtype=torch.float32)
        H.lib().call('srnn_segsum', H.ptr(dx0), D, B, Fr, D, H.ptr(dspk), st())
        dspkT = H.cast(dspk, T)
        dW_s = H.gemm(dspkT, spk_embT, transA=True)                  # (D, S)
        db_s = H.colsum(dspk, B, D)
        demb = H.gemm(dspkT, W_s)                                    # (B, S)
        dE = torch.zeros((S, S), device=dev, dtype=torch.float32)
        H.lib().call('srnn_index_add_rows', H.ptr(dE), S, S, H.ptr(spk_flat), B, S,
                     H.ptr(demb), S, st())
        grads += [dE]
        grads += nn.weight_grad_to_params(mod.spk_expand, dW_s.reshape(D, S, 1))
        grads += [db_s]
    for l in range(L):
        grads += g_rnn[l]
    grads += g_up + [g_up_b]
    dh0 = None
    if ctx.reset and need_h0:
        dh0 = torch.stack([H.colsum(dh_in[l], B, D) for l in range(L)], 0)
    return d_upper, dh0, grads


class SampleLevelMLP(torch.nn.Module):
    """model.py:266-325."""

    def __init__(self, frame_size, dim, q_levels, wnorm):
        super().__init__()
        self.q_levels = q_levels
        self.weight_norm = wnorm
        self.frame_size = frame_size
        self.dim = dim
        self.embedding = torch.nn.Embedding(q_levels, q_levels)
        self.input = torch.nn.Conv1d(q_levels, dim, kernel_size=frame_size, bias=False)
        init.kaiming_uniform_(self.input.weight)
        self.hidden = torch.nn.Conv1d(dim, dim, kernel_size=1)
        init.kaiming_uniform_(self.hidden.weight)
        init.constant_(self.hidden.bias, 0)
        self.output = torch.nn.Conv1d(dim, q_levels, kernel_size=1)
        nn.lecun_uniform(self.output.weight)
        init.constant_(self.output.bias, 0)
        if wnorm:
            nn.apply_weight_norm(self.input)
            nn.apply_weight_norm(self.hidden)
            nn.apply_weight_norm(self.output)

    def _param_list(self):
        return ([self.embedding.weight] + nn.weight_params(self.input) +
                nn.weight_params(self.hidden) + [self.hidden.bias] +
                nn.weight_params(self.output) + [self.output.bias])

    def tab(self, T):
        """Tab[k][q][:] = W_in[:, :, k] . E[q, :]  (FS0, Q, D): the folded embedding+conv."""
        return _build_tab(self, T)[0]

    def forward(self, prev_samples, upper_tier_conditioning):
        """model.py:308-325: indices (B, T+FS0-1), conditioning (B, T, D) -> log-probs (B,T,Q)."""
        H.need_cuda(upper_tier_conditioning)
        # (a window of the index stream is read in place: the kernels take a row stride)
        x = prev_samples.to(upper_tier_conditioning.device).long()
        if x.dim() != 2 or x.stride(1) != 1 or x.shape[1] != upper_tier_conditioning.shape[1] + \
                self.frame_size - 1:
            x = x.contiguous()
        u = upper_tier_conditioning
        if u.dtype not in (torch.float32, _dt(self)):
            u = u.float()
        # the registered op srnn::mlp_fwd (custom_ops.py; autograd: srnn::mlp_bwd)
        return custom_ops.mlp(x, u.contiguous(), self._param_list(), mlp_meta(self))


def _build_tab(mlp, T):
    Q, D, FS0 = mlp.q_levels, mlp.dim, mlp.frame_size
    W_in = nn.weight_of(mlp.input)                                       # (D, Q, FS0)
    Wp = H.permute3(W_in, (2, 0, 1), dtype=T)                            # (FS0, D, Q)
    ET = H.cast_param(mlp.embedding.weight, T)
    tab = torch.empty((FS0, Q, D), device=ET.device, dtype=T)
    H.gemm(ET, Wp, transB=True, out=tab, M=Q, N=D, K=Q, lda=Q, ldb=Q, ldc=D, batch=FS0, sA=0,
           sB=D * Q, sC=Q * D)
    return tab, Wp, ET


def mlp_forward(mlp, x, upper, ps):
    """SampleLevelMLP forward (model.py:308-325): (log-probs, state) (srnn::mlp_fwd)."""
    T = _dt(mlp)
    B, Tl, D = upper.shape
    Q, FS0 = mlp.q_levels, mlp.frame_size
    dev = upper.device
    tab, Wp, ET = _build_tab(mlp, T)
    a1 = torch.empty((B * Tl, D), device=dev, dtype=T)
    upper = upper.contiguous()
    # SRNN_MASK_BITS=1 (bf16): the ReLU masks of a1 and a2 leave the forward as bits, 16x
    # fewer bytes for the backward's masked GEMMs to read than the activations.  Off by
    # default: measured (MI355X, B = 128) the two masked dgrads gain 27 us each, but the
    # hidden GEMM's bit epilogue costs 26 us and the L1 gather's 2-B bit stores 87 us.
    bits = T == torch.bfloat16 and upper.dtype == T and D % 64 == 0 and \
        os.environ.get('SRNN_MASK_BITS', '0') != '0'
    # Default (bf16, D % 64 == 0): a1's mask alone leaves as bits, in the grouped layout
    # (u16 [D / 16][B T]): the da1 GEMM stages a tile's bits by LDS-DMA with its first
    # operand pieces instead of reading 2 B of a1 per output in its epilogue (SRNN_A1_BITS=0:
    # the bf16 mask).  The L1 kernel's 16-column workgroups write a column group's rows as
    # contiguous runs (the row-major layout's 2-B words of a row came from 64 workgroups).
    a1_bits = not bits and T == torch.bfloat16 and upper.dtype == T and D % 64 == 0 and \
        os.environ.get('SRNN_A1_BITS', '1') != '0'
    m1 = m2 = None
    ev = H.roof_begin()
    if bits:
        m1, m2 = H.relu_bits(B * Tl, D, dev), H.relu_bits(B * Tl, D, dev)
        H.lib().call('srnn_mlp_l1_bits', H.ptr(tab), H.ptr(x), x.stride(0), 0, B, Tl,
                     H.ptr(upper), D, H.ptr(a1), D, D, FS0, Q, H.ptr(m1), m1.stride(0),
                     H.stream())
    elif a1_bits:
        m1 = H.relu_bits_grouped(B * Tl, D, dev)
        H.lib().call('srnn_mlp_l1_bits', H.ptr(tab), H.ptr(x), x.stride(0), 0, B, Tl,
                     H.ptr(upper), D, H.ptr(a1), D, D, FS0, Q, H.ptr(m1), 0, H.stream())
    else:
        H.lib().call('srnn_mlp_l1', H.dcode(T), H.ptr(tab), H.ptr(x), x.stride(0), 0, B, Tl,
                     H.dcode(upper), H.ptr(upper), D, H.ptr(a1), D, D, FS0, Q, H.stream())
    # algorithmic bytes: upper read and a1 written once (+ its mask bits), the index windows
    H.roof_end('mlp_l1_gather', ev, B * Tl * D * (upper.element_size() + a1.element_size()) +
               (B * Tl * D // 8 if m1 is not None else 0) + B * (Tl + FS0 - 1) * 8)
    W_hid = _wcast(mlp.hidden, T).reshape(D, D)
    W_out = _wcast(mlp.output, T).reshape(Q, D)
    # bf16: the backward's activation-gradient GEMMs read W^T stored k-contiguous (the NT
    # shape of the pair-mode kernels: da1 1.43 -> 1.30 ms at B = 512, tools/da1_gemm_ab.py)
    W_t = (_wcast_t(mlp.hidden, T), _wcast_t(mlp.output, T)) if T == torch.bfloat16 else None
    ev = H.roof_begin()
    a2 = H.linear(a1, W_hid, bias=mlp.hidden.bias, relu=True, out_dtype=T, bits_out=m2)
    H.roof_end('mlp_hidden_gemm', ev, 2.0 * B * Tl * D * D)
    # bf16: the logits GEMM's epilogue applies the row log-softmax itself (its 256-column
    # tiles hold whole rows), so the (B T, Q) fp32 logits never round-trip through HBM
    # (SRNN_LSM_EPI=0: the separate logsoftmax pass)
    lsm = T == torch.bfloat16 and Q == 256 and os.environ.get('SRNN_LSM_EPI', '1') != '0'
    if lsm:
        H.lib().dll.srnn_gemm_logsoftmax_next()
    z = H.linear(a2, W_out, bias=mlp.output.bias)                    # (B*T, Q) fp32
    if lsm and H.lib().dll.srnn_gemm_logsoftmax_taken():
        logp = z
        _STATS['lsm_epi'] += 1
    else:
        logp = torch.empty((B * Tl, Q), device=dev, dtype=torch.float32)
        H.lib().call('srnn_logsoftmax_nll', H.ptr(z), Q, None, 0, Tl, B * Tl, Q, None,
                     H.ptr(logp), Q, None, H.F32, 0, 0.0, H.stream())
    ctx = _State()
    ctx.mlp = mlp
    ctx.T = T
    ctx.udt = upper.dtype
    ctx.dims = (B, Tl, D, Q, FS0)
    ctx.saved_tensors = (x, a1, a2, logp, Wp, ET, W_hid, W_out)
    ctx.bits = (m1, m2)
    ctx.W_t = W_t
    return logp.reshape(B, Tl, Q), ctx


def mlp_backward(ctx, dlogp, nll=None):
    """Backward of mlp_forward: (d_upper, [parameter gradients]).  nll = (target, T,
    gscale, g): the log-probs' gradient is sequence_nll_loss_bits' closed form (dlogp is then
    not read)."""
    mlp = ctx.mlp
    T = ctx.T
    B, Tl, D, Q, FS0 = ctx.dims
    x, a1, a2, logp, Wp, ET, W_hid, W_out = ctx.saved_tensors
    dev = logp.device
    st = H.stream
    M = B * Tl
    dz = torch.empty((M, Q), device=dev, dtype=T)
    if nll is not None:
        # loss gradient in closed form (custom_ops nll_bits): fused NLL + log-softmax
        # backward, dz = c (exp(logp) - onehot) straight into the GEMM operand dtype
        tg, Tt, gscale, gd = nll
        H.lib().call('srnn_nll_logsoftmax_bwd', H.ptr(tg), Tt, Tt, M, Q, H.ptr(logp), Q,
                     gscale, H.ptr(gd), H.ptr(dz), H.dcode(T), Q, st())
    else:
        dl = dlogp.reshape(M, Q).float().contiguous()
        H.lib().call('srnn_logsoftmax_bwd', H.ptr(dl), Q, H.ptr(logp), Q, M, Q, H.ptr(dz),
                     H.dcode(T), Q, st())
    dW_out = H.gemm(dz, a2, transA=True)                             # (Q, D)
    db_out = H.colsum(dz, M, Q)
    m1, m2 = ctx.bits
    ctx.bits = None
    W_t = ctx.W_t
    ctx.W_t = None
    # (M, D) = dz . W_out, through W_out^T (D, Q) when the forward made it
    Wo, tB = (W_t[1], True) if W_t is not None else (W_out, False)
    # bf16: the da2 GEMM's epilogue also sums its stored columns per 128-row block (the
    # hidden layer's bias gradient) -- one pass over da2 fewer than a separate column sum
    csp = None
    if T == torch.bfloat16 and M % 256 == 0 and os.environ.get('SRNN_CSUM_EPI', '1') != '0':
        csp = torch.empty((M // 128, D), device=dev, dtype=torch.float32)
        H.lib().call('srnn_gemm_csum_next', H.ptr(csp))
    ev = H.roof_begin()
    if m2 is not None:
        da2 = H.gemm(dz, Wo, transB=tB, mask_bits=m2, out_dtype=T)
    else:
        da2 = H.gemm(dz, Wo, transB=tB, mask=a2, out_dtype=T)
    H.roof_end('mlp_da2_gemm', ev, 2.0 * M * D * Q)
    if csp is not None and not H.lib().dll.srnn_gemm_csum_taken():
        csp = None
    if csp is not None:
        _STATS['csum_epi'] += 1
    ev = H.roof_begin()
    dW_hid = H.gemm(da2, a1, transA=True)                            # (D, D)
    H.roof_end('mlp_dw_hid_gemm', ev, 2.0 * M * D * D)
    db_hid = H.colsum(csp, M // 128, D) if csp is not None else H.colsum(da2, M, D)
    csp = None
    # d(upper) in upper's dtype: bf16 when the bottom tier hands the MLP a bf16 upper.  A
    # bf16 da1 also gets max |da1| from the GEMM's epilogue (the packed dTab scatter's
    # scale), so the scatter needs no pass of its own over da1
    amax = blk = None
    if ctx.udt == torch.bfloat16:
        amax = torch.zeros(1, device=dev, dtype=torch.int32)
        if FS0 == 16 and D % 256 == 0 and os.environ.get('SRNN_DTAB_BLK', '0') == '1':
            # ... and a column-blocked copy [D/4][M][4] of da1, the scatter's operand
            blk = torch.empty((D // 4, M, 4), device=dev, dtype=torch.bfloat16)
            H.lib().call('srnn_gemm_amax_blk_next', H.ptr(amax), H.ptr(blk))
        else:
            H.lib().call('srnn_gemm_amax_next', H.ptr(amax))
    Wh, tB = (W_t[0], True) if W_t is not None else (W_hid, False)
    ev = H.roof_begin()
    if m1 is not None:
        da1 = H.gemm(da2, Wh, transB=tB, mask_bits=m1, out_dtype=ctx.udt)     # (M, D)
    else:
        da1 = H.gemm(da2, Wh, transB=tB, mask=a1, out_dtype=ctx.udt)          # (M, D)
    H.roof_end('mlp_da1_gemm', ev, 2.0 * M * D * D)
    if amax is not None:
        taken = H.lib().dll.srnn_gemm_amax_taken()
        if taken != 2:
            blk = None
        if not taken:
            amax = None
    # folded embedding . conv backward: dTab[q][k][:] += da1[t] for x_{t+k} = q
    dtabT = torch.empty((Q, FS0 * D), device=dev, dtype=T)
    work = torch.empty(Q * FS0 * D, device=dev, dtype=torch.int64)
    # the same pass sums da1 over rows t = j (mod FS0): the bottom tier's upsampling bias
    # gradient (its output is this layer's `upper`), handed over on the returned gradient
    colsum = torch.empty(FS0 * D, device=dev, dtype=torch.float32)
    done = ctypes.c_int(0)
    ev = H.roof_begin()
    H.lib().call('srnn_mlp_dtab4', H.dcode(da1), H.ptr(da1), D, H.ptr(x), x.stride(0), 0, B,
                 Tl, H.ptr(dtabT), H.dcode(T), D, FS0, Q, H.ptr(work), work.numel() * 8,
                 H.ptr(colsum), ctypes.byref(done), H.ptr(amax), H.ptr(blk), st())
    blk = None
    # algorithmic bytes: da1 and the index window read once, dTab^T and the column sums
    # written once
    H.roof_end('dtab_scatter', ev, B * Tl * D * da1.element_size() +
               B * (Tl + FS0 - 1) * 8 + Q * FS0 * D * dtabT.element_size() + FS0 * D * 4)
    dE = H.gemm(dtabT, Wp.reshape(FS0 * D, Q))                       # (Q, Q)
    # dWp[k] = dTab[:, k]^T E for every tap k at once: (FS0 D, Q) = dtabT^T . ET, one GEMM
    # (the (FS0, D, Q) result is the same memory as the per-tap batch)
    dWp = torch.empty((FS0, D, Q), device=dev, dtype=torch.float32)
    H.gemm(dtabT, ET, transA=True, out=dWp, M=FS0 * D, N=Q, K=Q, lda=FS0 * D, ldb=Q, ldc=Q)
    dW_in = H.permute3(dWp, (1, 2, 0))                               # (D, Q, FS0)
    grads = [dE]
    grads += nn.weight_grad_to_params(mlp.input, dW_in)
    grads += nn.weight_grad_to_params(mlp.hidden, dW_hid.reshape(D, D, 1)) + [db_hid]
    grads += nn.weight_grad_to_params(mlp.output, dW_out.reshape(Q, D, 1)) + [db_out]
    d_upper = da1.reshape(B, Tl, D)
    if done.value:
        d_upper._srnn_colsum = (colsum, d_upper._version, FS0)
    return d_upper, grads


class Runner:
    """model.py:328-349."""

    def __init__(self, model):
        super().__init__()
        self.model = model
        self.reset_hidden_states()

    def reset_hidden_states(self):
        self.hidden_states = {rnn: None for rnn in self.model.frame_level_rnns}

    def run_rnn(self, rnn, prev_samples, upper_tier_conditioning, cond, spk, writer=None,
                iterations=None):
        (output, new_hidden) = rnn(prev_samples, upper_tier_conditioning,
                                   self.hidden_states[rnn], cond, spk, writer, iterations)
        self.hidden_states[rnn] = new_hidden.detach()    # TBPTT truncation (model.py:348)
        return output


class Predictor(Runner, torch.nn.Module):
    """model.py:352-436: teacher-forced forward with TBPTT hidden-state carry."""

    def __init__(self, model):
        super().__init__(model)

    def forward(self, input_sequences, reset, cond, spk, writer=None, iterations=None):
        if reset:
            self.reset_hidden_states()
        dev = next(self.model.parameters()).device
        H.need_cuda(torch.empty(0, device=dev))
        input_sequences = input_sequences.to(dev).long().contiguous()
        cond = cond.to(dev)
        spk = spk.to(dev)
        (batch_size, _) = input_sequences.size()
        (_, _, cond_dim) = cond.size()
        L = self.model.lookback
        q = self.model.q_levels
        mode = 0 if self.model.ulaw else 1
        upper = None
        for rnn in reversed(self.model.frame_level_rnns):
            n = rnn.n_frame_samples
            seg = input_sequences[:, L - n: input_sequences.shape[1] - n + 1]
            prev = utils._dequant(seg, q, 2.0, mode)                    # 2 * dequantize
            prev = prev.view(batch_size, -1, n)
            if upper is None:
                c = cond.contiguous().view(batch_size, -1, cond_dim)
                s = spk.contiguous().view(batch_size, -1)
                upper = self.run_rnn(rnn, prev, None, c, s, writer, iterations)
            else:
                upper = self.run_rnn(rnn, prev, upper, None, None, writer, iterations)
        fs0 = self.model.frame_level_rnns[0].frame_size
        return self.model.sample_level_mlp(input_sequences[:, L - fs0:], upper)


def generation_weights(model, dtype=None):
    """Folded, device-resident weight layouts for srnn::generate (weight-norm applied once):
    (tensors, meta) -- srnn_model_struct(tensors, meta) rebuilds the C ABI's SrnnModel."""
    T = dtype or model.compute_dtype
    D = model.dim
    ws = []
    meta = [len(model.frame_level_rnns), model.n_rnn, D, model.q_levels, model.cond_dim,
            H.dcode(T)]
    with torch.no_grad():
        for k, rnn in enumerate(model.frame_level_rnns):
            nfs = rnn.n_frame_samples
            W_ie = nn.weight_of(rnn.input_expand).reshape(D, nfs)
            if rnn.is_cond:
                C = model.cond_dim
                W_c = nn.weight_of(rnn.cond_expand).reshape(D, C)
                w_in = torch.empty((D, nfs + C), device=W_ie.device, dtype=T)
                H.lib().call('srnn_copy2d', H.F32, H.dcode(T), D, nfs, H.ptr(W_ie.contiguous()),
                             nfs, H.ptr(w_in), nfs + C, H.stream())
                H.lib().call('srnn_copy2d', H.F32, H.dcode(T), D, C, H.ptr(W_c.contiguous()), C,
                             H.ptr(w_in[:, nfs:]), nfs + C, H.stream())
                meta += [rnn.frame_size, nfs, nfs + C, 0]
                ws.append(w_in)
            else:
                meta += [rnn.frame_size, nfs, nfs, 1]
                ws += [H.cast(W_ie.contiguous(), T), rnn.input_expand.bias.detach().contiguous()]
            for l in range(model.n_rnn):
                ws += [H.cast(getattr(rnn.rnn, 'weight_ih_l%d' % l).detach().contiguous(), T),
                       H.cast(getattr(rnn.rnn, 'weight_hh_l%d' % l).detach().contiguous(), T),
                       getattr(rnn.rnn, 'bias_ih_l%d' % l).detach().contiguous(),
                       getattr(rnn.rnn, 'bias_hh_l%d' % l).detach().contiguous()]
            k_ = rnn.frame_size
            ws += [nn.convt_operand(rnn.upsampling.conv_t, T),
                   H.permute3(rnn.upsampling.bias.detach().reshape(1, D, k_), (0, 2, 1)),
                   rnn.h0.detach().float().contiguous()]
        mlp = model.sample_level_mlp
        ws += [mlp.tab(T), H.cast(nn.weight_of(mlp.hidden).reshape(D, D).contiguous(), T),
               mlp.hidden.bias.detach().contiguous(),
               H.cast(nn.weight_of(mlp.output).reshape(model.q_levels, D).contiguous(), T),
               mlp.output.bias.detach().contiguous()]
    meta.append(model.lookback)
    return ws, meta


def srnn_model_struct(ws, meta):
    """The C ABI's SrnnModel (include/samplernn_hip.h) over generation_weights' tensors."""
    m = H.SrnnModel()
    m.n_tiers, m.n_rnn, m.dim, m.q_levels, m.cond_dim, m.dtype = [int(v) for v in meta[:6]]
    it = iter(ws)
    for k in range(m.n_tiers):
        t = m.tier[k]
        t.frame_size, t.n_frame_samples, t.in_dim, has_b = [int(v) for v in
                                                            meta[6 + 4 * k: 10 + 4 * k]]
        t.w_in = H.ptr(next(it))
        if has_b:
            t.b_in = H.ptr(next(it))
        for l in range(m.n_rnn):
            t.w_ih[l], t.w_hh[l] = H.ptr(next(it)), H.ptr(next(it))
            t.b_ih[l], t.b_hh[l] = H.ptr(next(it)), H.ptr(next(it))
        t.w_up, t.b_up, t.h0 = H.ptr(next(it)), H.ptr(next(it)), H.ptr(next(it))
    m.tab, m.w_hid, m.b_hid = H.ptr(next(it)), H.ptr(next(it)), H.ptr(next(it))
    m.w_out, m.b_out = H.ptr(next(it)), H.ptr(next(it))
    return m


def top_row_bias(model, spk):
    """(n_seqs, D): spk_expand(spk_embedding(spk)) + b_spk + b_cond + b_in for the top tier."""
    top = model.frame_level_rnns[-1]
    D, S = model.dim, model.spk_dim
    dev = spk.device
    with torch.no_grad():
        n = spk.numel()
        emb = torch.empty((n, S), device=dev, dtype=torch.float32)
        H.lib().call('srnn_gather_rows', H.ptr(top.spk_embedding.weight), S,
                     H.ptr(spk.reshape(-1).contiguous()), n, S, H.ptr(emb), H.F32, S, H.stream())
        bias = torch.empty(D, device=dev, dtype=torch.float32)
        H.lib().call('srnn_axpby', H.ptr(bias), H.ptr(top.spk_expand.bias),
                     H.ptr(top.cond_expand.bias), 1.0, 1.0, D, H.stream())
        H.lib().call('srnn_axpby', H.ptr(bias), H.ptr(bias), H.ptr(top.input_expand.bias), 1.0,
                     1.0, D, H.stream())
        W_s = nn.weight_of(top.spk_expand).reshape(D, S).contiguous()
        return H.linear(emb, W_s, bias=bias)


class Generator(Runner):
    """model.py:439-520: autoregressive generation, the whole loop on the device.

    __call__(n_seqs, seq_len, cond, spk) keeps the reference contract: `seq_len` is
    ignored (recomputed as num_cond * lookback, model.py:455), `cond` is a (num_cond, C)
    array shared by all rows (or (n_seqs, num_cond, C) per row), `spk` an int (or one per
    row), and the result is a host float32 (n_seqs, num_cond * lookback) tensor of
    dequantized samples.  Sampling is argmax(p / q), q ~ Exp(1), exactly what torch>=2's
    CPU `multinomial(1)` computes: sampler='torch' draws q from torch's CPU generator in
    the reference's order (bit-replay of the reference stream); sampler='philox' draws q
    on the device (counter-based Philox4x32-10, seed) for long runs.  `cuda` is accepted
    for API compatibility; the product path always runs on the GPU.  persistent=True (the
    default) runs the sample chain between bottom-tier ticks as one persistent launch
    (gen_mlp.hip) where the shape fits, else per-sample kernels.
    """

    def __init__(self, model, cuda=False):
        super().__init__(model)
        self.cuda = cuda
        self.last_sequences = None

    def __call__(self, n_seqs, seq_len, cond, spk, sampler='torch', seed=0, noise=None,
                 return_logp=False, use_graph=True, dtype=None, persistent=True, row_offset=0):
        """row_offset: these n_seqs rows are rows [row_offset, row_offset + n_seqs) of a larger
        batch (rank-sharded generation, see shard_generate): the Philox noise (sampler='philox')
        is that of the global rows, so shards reproduce the single-process stream."""
        model = self.model
        self.reset_hidden_states()
        dev = next(model.parameters()).device
        H.need_cuda(torch.empty(0, device=dev))
        cond = torch.as_tensor(np.asarray(cond) if not torch.is_tensor(cond) else cond)
        if cond.dim() == 2:
            cond = cond.unsqueeze(0).expand(n_seqs, *cond.shape)
        cond = cond.to(dev, torch.float32).contiguous()
        num_cond = cond.shape[1]
        spk = torch.as_tensor(np.asarray(spk) if not torch.is_tensor(spk) else spk).reshape(-1)
        if spk.numel() == 1:
            spk = spk.expand(n_seqs)
        spk = spk.to(dev, torch.long).contiguous()
        L = model.lookback
        T = num_cond * L
        Q = model.q_levels
        weights, meta = generation_weights(model, dtype)
        row_bias = top_row_bias(model, spk)
        if noise is None and sampler == 'torch':
            noise = torch.empty(T, n_seqs, Q).exponential_(1)
        if noise is not None:
            noise = torch.as_tensor(noise).to(dev, torch.float32).contiguous()
            assert noise.shape == (T, n_seqs, Q), 'noise must be (T, n_seqs, Q)'
        # the registered op srnn::generate (custom_ops.py): the whole sample loop on the device
        with torch.no_grad():
            seq, logp = torch.ops.srnn.generate(
                weights, meta, cond, row_bias, noise, int(seed) & ((1 << 63) - 1),
                int(row_offset), (1 if use_graph else 0) | (0 if persistent else 2),
                bool(return_logp))
        assert utils.q_zero(Q) == Q // 2
        self.last_sequences = seq
        out = model.dequantize(seq[:, L:], Q).cpu()
        if return_logp:
            return out, logp.permute(1, 0, 2).contiguous()
        return out


def shard_generate(generator, n_seqs, cond, spk, seed, rank=None, world=None, sampler='philox',
                   seq_len=0, noise_rows=None, **kw):
    """Rank-sharded generation (the reference runs generate.py:241-253 per file on
    one device): rank r generates the contiguous rows [r n / N, (r + 1) n / N) of an n_seqs batch
    with replicated weights and no collective in the loop; the dequantized rows are gathered to
    every rank at the end, and the union equals the single-process output for either sampler:
      * 'philox': the device noise of the GLOBAL rows (row_offset);
      * 'torch' (the reference's multinomial stream, model.py:514-517): every rank draws the
        whole batch's Exp(1) noise from torch's CPU generator exactly as a single process
        would (one (T, n_seqs, Q) draw, so every rank must have been seeded alike) and keeps
        its rows' slice -- host memory T * n_seqs * Q * 4 bytes per rank.  noise_rows: the
        caller's true row count when n_seqs includes padding rows (to a multiple of the world
        size): the draw is then (T, noise_rows, Q), as the unpadded single-process run makes
        it, and the padding rows get unit noise (their output is discarded).
    cond: (num_cond, C) shared or (n_seqs, num_cond, C) per row; spk: int or (n_seqs,).
    seq_len is accepted like Generator's (the reference ignores it, model.py:455).
    Returns the host float32 (n_seqs, num_cond * lookback) batch."""
    import distributed as Dd
    rank = Dd.rank() if rank is None else rank
    world = Dd.world() if world is None else world
    if sampler not in ('philox', 'torch'):
        raise ValueError('shard_generate: unknown sampler %r' % (sampler,))
    rows = Dd.shard_rows(n_seqs, rank, world)
    c = torch.as_tensor(np.asarray(cond) if not torch.is_tensor(cond) else cond)
    num_cond = c.shape[-2]
    if c.dim() == 3:
        c = c[rows]
    s = torch.as_tensor(np.asarray(spk) if not torch.is_tensor(spk) else spk).reshape(-1)
    if s.numel() > 1:
        s = s[rows]
    if sampler == 'torch' and kw.get('noise') is None:
        model = generator.model
        nr = n_seqs if noise_rows is None else int(noise_rows)
        if not 0 < nr <= n_seqs:
            raise ValueError('shard_generate: noise_rows %d outside (0, %d]' % (nr, n_seqs))
        full = torch.empty(num_cond * model.lookback, nr, model.q_levels).exponential_(1)
        if nr < n_seqs:
            full = torch.cat([full, full.new_ones((full.shape[0], n_seqs - nr, full.shape[2]))],
                             1)
        kw['noise'] = full[:, rows].contiguous()
        del full
    out = generator(rows.stop - rows.start, seq_len, c, s, sampler=sampler, seed=seed,
                    row_offset=rows.start, **kw)
    return Dd.gather_rows(out, n_seqs)
