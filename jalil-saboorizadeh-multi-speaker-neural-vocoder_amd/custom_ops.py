"""torch.library registration of the HIP operators ("registered as torch.library
custom ops, wrapped by the new model.py classes").

The drop-in classes call these ops, so the registered ops ARE the product path:

  srnn::tier_fwd / tier_bwd     FrameLevelRNN.forward (model.py:180-263) and its backward:
                                input / cond / speaker projections, the GRU sweep(s),
                                LearnedUpsampling1d -- model.tier_forward / tier_backward
  srnn::mlp_fwd / mlp_bwd       SampleLevelMLP.forward (model.py:308-325) + log_softmax
  srnn::nll_bits / nll_bits_bwd sequence_nll_loss_bits (nn.py:66-70); its backward hands the
                                MLP the gradient in closed form (fused NLL + log-softmax)
  srnn::upsample / upsample_bwd LearnedUpsampling1d used on its own (nn.py:7-43)
  srnn::dequant                 2 * udequantize / linear_dequantize (utils.py:18-19, 62-63)
  srnn::adam_clip_              gradient_clipping + Adam (optim.py:4-21), in place
  srnn::step_advance_           the device step counters srnn::adam_clip_ can read (graph mode)
  srnn::generate                Generator.__call__'s sample loop (model.py:445-520)

Every op has a fake (meta) kernel, so FakeTensor / torch.compile tracing sees shapes without
running HIP code, and the differentiable ones have their autograd formula attached with
torch.library.register_autograd (backward = the *_bwd op).

Saved activations: a forward op returns, beside its outputs, a 0-element int64 host `handle`;
the activations its backward needs (bf16 operand copies, GRU gates, MLP a1 / a2 / log-probs)
stay in a per-call stash keyed by that handle and are released with the handle (when autograd
frees the graph, or at once under no_grad).  The backward op takes the handle.  This keeps the
forward outputs free of aliasing with inputs (custom ops may not return views of their inputs,
and many saved tensors are the fp32 parameters themselves in the fp32 mode) without copying.
"""
import weakref
from typing import Optional

import torch
from torch import Tensor

import samplernn_hip as H

_STASH = {}
_NEXT = [1]


def _stash(state):
    """A 0-element int64 host tensor standing for `state` (its key rides as an attribute of
    the tensor object, so the handle has no data: equal across runs for every comparison)."""
    key = _NEXT[0]
    _NEXT[0] += 1
    _STASH[key] = state
    handle = torch.empty(0, dtype=torch.int64)
    handle._srnn_key = key
    weakref.finalize(handle, _STASH.pop, key, None)
    return handle


def _take(handle):
    st = _STASH.get(getattr(handle, '_srnn_key', None))
    if st is None:
        raise RuntimeError('srnn: saved state of this forward is gone (backward run twice '
                           'without retain_graph, or the handle was dropped)')
    return st


def _empty():
    return torch.empty(0)


def _opt(t):
    return None if t is None or t.numel() == 0 else t


# ------------------------------------------------------------------ FrameLevelRNN
@torch.library.custom_op('srnn::tier_fwd', mutates_args=())
def tier_fwd(prev: Tensor, upper: Optional[Tensor], cond: Optional[Tensor],
             spk: Optional[Tensor], hidden: Optional[Tensor], h0: Tensor, params: list[Tensor],
             meta: list[int]) -> tuple[Tensor, Tensor, Tensor]:
    import model
    spec = model.TierSpec(meta, params)
    y, h_new, st = model.tier_forward(spec, prev, upper, cond, spk, hidden, h0, params)
    return y, h_new, _stash(st)


@tier_fwd.register_fake
def _(prev, upper, cond, spk, hidden, h0, params, meta):
    B, Fr, _ = prev.shape
    D, k, L, feeds, dt = meta[0], meta[2], meta[3], meta[5], meta[6]
    ydt = torch.bfloat16 if (feeds and dt) else torch.float32
    return (prev.new_empty((B, Fr * k, D), dtype=ydt),
            prev.new_empty((L, B, D), dtype=torch.float32),
            torch.empty(0, dtype=torch.int64, device='cpu'))


@torch.library.custom_op('srnn::tier_bwd', mutates_args=())
def tier_bwd(dy: Tensor, handle: Tensor, params: list[Tensor], meta: list[int], need_h0: bool,
             has_upper: bool) -> list[Tensor]:
    """[d_upper (B, F, D) fp32 | empty, dh0 (n_rnn, D) | empty, *parameter gradients
    (_param_list order)]."""
    import model
    d_upper, dh0, grads = model.tier_backward(_take(handle), dy, need_h0)
    return [d_upper if has_upper else _empty().to(dy.device),
            dh0 if need_h0 else _empty().to(dy.device)] + list(grads)


@tier_bwd.register_fake
def _(dy, handle, params, meta, need_h0, has_upper):
    B, FK, D = dy.shape
    k, L = meta[2], meta[3]
    return [dy.new_empty((B, FK // k, D), dtype=torch.float32) if has_upper else dy.new_empty(0),
            dy.new_empty((L, D), dtype=torch.float32) if need_h0 else dy.new_empty(0)] + \
        [torch.empty_like(p) for p in params]


def _tier_setup(ctx, inputs, output):
    prev, upper, cond, spk, hidden, h0, params, meta = inputs
    ctx.has_upper = upper is not None
    ctx.need_h0 = hidden is None and h0.requires_grad
    ctx.nparams = len(params)
    ctx.params = params
    ctx.meta = meta
    ctx.save_for_backward(output[2])
    ctx.mark_non_differentiable(output[1], output[2])


def _tier_backward(ctx, dy, dh_new, dhandle):
    (handle,) = ctx.saved_tensors
    out = torch.ops.srnn.tier_bwd(dy.contiguous(), handle, ctx.params, ctx.meta, ctx.need_h0,
                                  ctx.has_upper)
    d_upper = out[0] if ctx.has_upper else None
    dh0 = out[1] if ctx.need_h0 else None
    return None, d_upper, None, None, None, dh0, list(out[2:]), None


tier_fwd.register_autograd(_tier_backward, setup_context=_tier_setup)


def tier(prev, upper, cond, spk, hidden, h0, params, meta):
    """(conditioning for the tier below (B, F * k, D), new hidden (n_rnn, B, D))."""
    y, h_new, _ = torch.ops.srnn.tier_fwd(prev, upper, cond, spk, hidden, h0, params, meta)
    return y, h_new


# ------------------------------------------------------------------ SampleLevelMLP
@torch.library.custom_op('srnn::mlp_fwd', mutates_args=())
def mlp_fwd(x: Tensor, upper: Tensor, params: list[Tensor],
            meta: list[int]) -> tuple[Tensor, Tensor]:
    import model
    logp, st = model.mlp_forward(model.MlpSpec(meta, params), x, upper, params)
    return logp, _stash(st)


@mlp_fwd.register_fake
def _(x, upper, params, meta):
    B, Tl, _ = upper.shape
    return (upper.new_empty((B, Tl, meta[0]), dtype=torch.float32),
            torch.empty(0, dtype=torch.int64, device='cpu'))


@torch.library.custom_op('srnn::mlp_bwd', mutates_args=())
def mlp_bwd(dlogp: Tensor, handle: Tensor, params: list[Tensor], meta: list[int],
            upper_bf16: bool, nll_target: Optional[Tensor], nll_scale: float,
            nll_g: Optional[Tensor]) -> list[Tensor]:
    """[d_upper, *parameter gradients].  nll_target given: the log-probs' gradient is
    sequence_nll_loss_bits' closed form -nll_scale * nll_g * onehot(target) (dlogp unread)."""
    import model
    nll = None
    if nll_target is not None:
        nll = (nll_target, nll_target.shape[1], nll_scale, nll_g)
    d_upper, grads = model.mlp_backward(_take(handle), dlogp, nll)
    return [d_upper] + list(grads)


@mlp_bwd.register_fake
def _(dlogp, handle, params, meta, upper_bf16, nll_target, nll_scale, nll_g):
    B, Tl, _ = dlogp.shape
    udt = torch.bfloat16 if upper_bf16 else torch.float32
    return [dlogp.new_empty((B, Tl, meta[1]), dtype=udt)] + [torch.empty_like(p) for p in params]


class FusedNllToken:
    """Marks the MLP's log-prob output so the NLL backward can hand the MLP its loss gradient
    in closed form instead of a dense (B, T, Q) fp32 tensor; `emitted` records that it did,
    so the MLP backward can refuse a placeholder that autograd summed with another gradient
    (log-probs used twice) instead of computing a wrong result."""
    __slots__ = ('emitted',)

    def __init__(self):
        self.emitted = False


def _mlp_setup(ctx, inputs, output):
    x, upper, params, meta = inputs
    ctx.params = params
    ctx.meta = meta
    ctx.upper_bf16 = upper.dtype == torch.bfloat16
    ctx.save_for_backward(output[1])
    ctx.mark_non_differentiable(output[1])
    ctx.tok = FusedNllToken()
    output[0]._srnn_nll_token = ctx.tok


def _mlp_backward(ctx, dlogp, dhandle):
    (handle,) = ctx.saved_tensors
    nll = getattr(dlogp, '_srnn_nll', None)
    if nll is None and ctx.tok.emitted:
        raise RuntimeError('the fused NLL gradient of the MLP log-probs was combined with '
                           'another gradient (log-probs used twice); run with SRNN_FUSED_NLL=0')
    if nll is not None:
        out = torch.ops.srnn.mlp_bwd(dlogp, handle, ctx.params, ctx.meta, ctx.upper_bf16,
                                     nll[0], nll[1], nll[2])
    else:
        out = torch.ops.srnn.mlp_bwd(dlogp, handle, ctx.params, ctx.meta, ctx.upper_bf16, None,
                                     0.0, None)
    return None, out[0], list(out[1:]), None


mlp_fwd.register_autograd(_mlp_backward, setup_context=_mlp_setup)


def mlp(x, upper, params, meta):
    logp, _ = torch.ops.srnn.mlp_fwd(x, upper, params, meta)
    return logp


# ------------------------------------------------------------------ NLL in bits
@torch.library.custom_op('srnn::nll_bits', mutates_args=())
def nll_bits(logp: Tensor, target: Tensor) -> Tensor:
    import nn
    B, T, Q = logp.shape
    lp = logp.contiguous()
    tg = target.reshape(B, T).contiguous()
    rows = torch.empty(B * T, device=lp.device, dtype=torch.float32)
    H.lib().call('srnn_nll_fwd', H.ptr(lp), Q, H.ptr(tg), T, T, B * T, H.ptr(rows), H.stream())
    return H.colsum(rows, B * T, 1, alpha=nn.LOG2E / (B * T)).reshape(())


@nll_bits.register_fake
def _(logp, target):
    return logp.new_empty((), dtype=torch.float32)


@torch.library.custom_op('srnn::nll_bits_bwd', mutates_args=())
def nll_bits_bwd(g: Tensor, target: Tensor, B: int, T: int, Q: int, dense: bool) -> Tensor:
    """dense: the (B, T, Q) fp32 gradient -g log2(e)/N onehot(target); else a zero
    placeholder (the MLP consumes the closed form, mlp_bwd's nll_* arguments)."""
    import nn
    if not dense:
        return torch.zeros((), device=target.device, dtype=torch.float32).expand(B, T, Q)
    tg = target.reshape(B, T).contiguous()
    gd = g.detach().float().reshape(1).contiguous()
    d = torch.empty((B, T, Q), device=tg.device, dtype=torch.float32)
    H.lib().call('srnn_nll_bwd', H.ptr(tg), T, T, B * T, Q, H.ptr(d), Q, nn.LOG2E / (B * T),
                 H.ptr(gd), H.stream())
    return d


@nll_bits_bwd.register_fake
def _(g, target, B, T, Q, dense):
    return target.new_empty((B, T, Q), dtype=torch.float32)


def _nll_setup(ctx, inputs, output):
    logp, target = inputs
    ctx.shape = tuple(logp.shape)
    ctx.save_for_backward(target)
    import nn
    tok = getattr(logp, '_srnn_nll_token', None)
    # (the closed-form hand-over relies on Python attributes travelling with the gradient:
    #  eager autograd only, never while a compiler traces the backward)
    ctx.tok = tok if (nn.FUSED_NLL and isinstance(tok, FusedNllToken) and ctx.shape[2] == 256
                      and not torch.compiler.is_compiling()) else None


def _nll_backward(ctx, g):
    import nn
    (target,) = ctx.saved_tensors
    B, T, Q = ctx.shape
    d = torch.ops.srnn.nll_bits_bwd(g, target, B, T, Q, ctx.tok is None)
    if ctx.tok is not None:
        tg = target.reshape(B, T).contiguous()
        d._srnn_nll = (tg, nn.LOG2E / (B * T), g.detach().float().reshape(1).contiguous())
        ctx.tok.emitted = True
    return d, None


nll_bits.register_autograd(_nll_backward, setup_context=_nll_setup)


# ------------------------------------------------------------------ LearnedUpsampling1d
@torch.library.custom_op('srnn::upsample', mutates_args=())
def upsample(x: Tensor, params: list[Tensor], k: int, weight_norm: bool,
             has_bias: bool) -> tuple[Tensor, Tensor]:
    import nn
    out, st = nn.upsample_forward(x, params, k, weight_norm, has_bias)
    return out, _stash(st)


@upsample.register_fake
def _(x, params, k, weight_norm, has_bias):
    B, Cin, Lx = x.shape
    v = params[1] if weight_norm else params[0]
    return (x.new_empty((B, v.shape[1], Lx * k), dtype=torch.float32),
            torch.empty(0, dtype=torch.int64, device='cpu'))


@torch.library.custom_op('srnn::upsample_bwd', mutates_args=())
def upsample_bwd(dout: Tensor, handle: Tensor, params: list[Tensor], k: int,
                 weight_norm: bool) -> list[Tensor]:
    import nn
    dx, grads = nn.upsample_backward(_take(handle), dout)
    return [dx] + list(grads)


@upsample_bwd.register_fake
def _(dout, handle, params, k, weight_norm):
    B, _, LK = dout.shape
    cin = (params[1] if weight_norm else params[0]).shape[0]
    return [dout.new_empty((B, cin, LK // k), dtype=torch.float32)] + \
        [torch.empty_like(p) for p in params]


def _up_setup(ctx, inputs, output):
    ctx.params = inputs[1]
    ctx.k, ctx.wn = inputs[2], inputs[3]
    ctx.save_for_backward(output[1])
    ctx.mark_non_differentiable(output[1])


def _up_backward(ctx, dout, dhandle):
    (handle,) = ctx.saved_tensors
    out = torch.ops.srnn.upsample_bwd(dout.contiguous(), handle, ctx.params, ctx.k, ctx.wn)
    return out[0], list(out[1:]), None, None, None


upsample.register_autograd(_up_backward, setup_context=_up_setup)


# ------------------------------------------------------------------ mu-law dequantisation
@torch.library.custom_op('srnn::dequant', mutates_args=())
def dequant(samples: Tensor, q_levels: int, scale: float, mode: int) -> Tensor:
    """scale * (udequantize (mode 0) | linear_dequantize (mode 1)) of int64 indices."""
    import utils
    return utils._dequant_impl(samples, q_levels, scale, mode)


@dequant.register_fake
def _(samples, q_levels, scale, mode):
    return samples.new_empty(samples.shape, dtype=torch.float32)


# ------------------------------------------------------------------ clip + Adam
@torch.library.custom_op('srnn::adam_clip_',
                         mutates_args=('params', 'grads', 'exp_avg', 'exp_avg_sq', 'shadows'))
def adam_clip_(params: list[Tensor], grads: list[Optional[Tensor]], exp_avg: list[Tensor],
               exp_avg_sq: list[Tensor], shadows: list[Optional[Tensor]], grad_scale: float,
               clip_lo: float, clip_hi: float, lr: float, beta1: float, beta2: float,
               eps: float, step: int, dstep: Optional[Tensor] = None) -> None:
    """gradient_clipping(lo, hi) + torch.optim.Adam over every tensor in ONE launch per 64
    (srnn_adam_clip_multi3): g = clamp(g * grad_scale) (written back for fp32 gradients),
    moments and parameters updated in place, bf16 shadows (optional) refreshed; a None
    gradient is an all-zero one; skipped on the device while the persistent-sweep failure
    flag is up.  All gradients share one dtype (fp32, or bf16 from DP buckets).  dstep: a
    one-element int64 device tensor holding the count of completed steps, read by the
    kernel in place of `step` (a graph-replayed step; advanced by srnn::step_advance_)."""
    import ctypes
    n = len(params)
    if n == 0:
        return
    if dstep is not None and (dstep.dtype != torch.int64 or dstep.numel() < 1 or
                              dstep.device != params[0].device):
        raise ValueError('adam_clip_: dstep must be an int64 tensor on the parameters\' device')
    arr = lambda ts: (ctypes.c_void_p * n)(*[H.ptr(t) for t in ts])  # noqa: E731
    gdt = next((g.dtype for g in grads if g is not None), torch.float32)
    H.lib().call('srnn_adam_clip_multi3', n, arr(params), arr(grads), H.dcode(gdt),
                 float(grad_scale), arr(exp_avg), arr(exp_avg_sq),
                 arr(shadows) if any(t is not None for t in shadows) else None,
                 (ctypes.c_int64 * n)(*[p.numel() for p in params]), float(clip_lo),
                 float(clip_hi), float(lr), float(beta1), float(beta2), float(eps), int(step),
                 H.ptr(dstep) if dstep is not None else None, H.stream())


@adam_clip_.register_fake
def _(params, grads, exp_avg, exp_avg_sq, shadows, grad_scale, clip_lo, clip_hi, lr, beta1,
      beta2, eps, step, dstep=None):
    return None


@torch.library.custom_op('srnn::step_advance_', mutates_args=('dstep',))
def step_advance_(dstep: Tensor) -> None:
    """Device step counters += 1 unless the persistent-sweep failure flag is up
    (srnn_step_advance): the count srnn::adam_clip_ reads when given dstep."""
    if dstep.dtype != torch.int64 or not dstep.is_contiguous():
        raise ValueError('step_advance_: contiguous int64 counters')
    H.lib().call('srnn_step_advance', H.ptr(dstep), dstep.numel(), H.stream())


@step_advance_.register_fake
def _(dstep):
    return None


# ------------------------------------------------------------------ generation
@torch.library.custom_op('srnn::generate', mutates_args=())
def generate(weights: list[Tensor], meta: list[int], cond: Tensor, row_bias: Tensor,
             noise: Optional[Tensor], seed: int, row_offset: int, flags: int,
             return_logp: bool) -> tuple[Tensor, Tensor]:
    """The whole autoregressive loop (model.py:445-520) on the device: (sample indices
    (n_seqs, L + T) int64, per-step log-probs (T, n_seqs, Q) or empty).  weights / meta:
    model.generation_weights' tensors and layout."""
    import ctypes
    import model
    m = model.srnn_model_struct(weights, meta)
    n_seqs, num_cond = cond.shape[0], cond.shape[1]
    L = m.tier[m.n_tiers - 1].n_frame_samples
    T = num_cond * L
    Q = m.q_levels
    dev = cond.device
    seq = torch.full((n_seqs, L + T), Q // 2, dtype=torch.long, device=dev)   # q_zero
    logp = torch.empty((T, n_seqs, Q), device=dev) if return_logp else torch.empty(0, device=dev)
    sz = ctypes.c_size_t(0)
    H.lib().call('srnn_gen_workspace_size', ctypes.byref(m), n_seqs, ctypes.byref(sz))
    ws = torch.empty(sz.value, device=dev, dtype=torch.uint8)
    H.lib().call('srnn_generate2', ctypes.byref(m), n_seqs, num_cond, H.ptr(cond),
                 H.ptr(row_bias), H.ptr(noise), int(seed) & ((1 << 64) - 1), int(row_offset),
                 H.ptr(seq), H.ptr(logp) if return_logp else None, H.ptr(ws), sz.value,
                 int(flags), H.stream())
    return seq, logp


@generate.register_fake
def _(weights, meta, cond, row_bias, noise, seed, row_offset, flags, return_logp):
    n_seqs, num_cond = cond.shape[0], cond.shape[1]
    L = meta[-1]
    Q = meta[3]                      # q_levels (model.generation_weights' meta layout)
    T = num_cond * L
    return (cond.new_empty((n_seqs, L + T), dtype=torch.long),
            cond.new_empty((T, n_seqs, Q) if return_logp else (0,)))


OPS = ('tier_fwd', 'tier_bwd', 'mlp_fwd', 'mlp_bwd', 'nll_bits', 'nll_bits_bwd', 'upsample',
       'upsample_bwd', 'dequant', 'adam_clip_', 'step_advance_', 'generate')
