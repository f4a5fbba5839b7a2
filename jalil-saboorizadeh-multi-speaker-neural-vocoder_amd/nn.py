"""Drop-in for the reference's nn.py (nn.py:1-70).

LearnedUpsampling1d keeps the reference's parameters (conv_t = ConvTranspose1d with
stride = kernel_size, plus a per-(channel, position) bias) and computes on the HIP
GEMM; sequence_nll_loss_bits runs the HIP NLL kernels.  The init helpers are the
reference's recipes (they only touch host tensors at construction time).
"""
import math
import os

import torch
from torch import nn

import samplernn_hip as H

LOG2E = math.log(math.e, 2)


def weight_of(mod):
    """Effective weight of a conv/linear container: weight, or g * v / ||v|| when the
    module carries weight_g / weight_v (torch weight_norm naming, dim=0)."""
    if hasattr(mod, 'weight_g'):
        return H.weight_norm(mod.weight_g, mod.weight_v)
    return mod.weight


def weight_grad_to_params(mod, dw):
    """Map a gradient w.r.t. the effective weight to the module's parameters, in the
    order returned by weight_params(mod)."""
    if hasattr(mod, 'weight_g'):
        return list(H.weight_norm_bwd(mod.weight_g, mod.weight_v, dw))
    return [dw]


def convt_operand(conv_t, dtype):
    """GEMM operand of a ConvTranspose1d weight (Cin, Cout, k): W (k, Cout, Cin) in `dtype`,
    the weight norm (when present) folded in on the device without an fp32 weight."""
    v = conv_t.weight_v if hasattr(conv_t, 'weight_g') else conv_t.weight
    Cin, Cout, k = v.shape
    if H.convt_operand_ok(Cin, Cout, k):
        g = conv_t.weight_g if hasattr(conv_t, 'weight_g') else None
        return H.convt_operand(g, v, k, dtype)
    return H.permute3(weight_of(conv_t), (2, 1, 0), dtype=dtype)


def convt_grad_to_params(conv_t, dwt):
    """Parameter gradients of a ConvTranspose1d weight from the transposed GEMM weight
    gradient dwt (Cin, k * Cout) = [i][j * Cout + o]."""
    v = conv_t.weight_v if hasattr(conv_t, 'weight_g') else conv_t.weight
    Cin, Cout, k = v.shape
    if hasattr(conv_t, 'weight_g') and Cout % 4 == 0 and k * (Cout + 4) * 4 <= 150 * 1024:
        return list(H.convt_wn_bwd(conv_t.weight_g, v, dwt, k))
    dw = H.permute3(dwt.reshape(Cin, k, Cout), (0, 2, 1))            # (Cin, Cout, k)
    return weight_grad_to_params(conv_t, dw)


def weight_params(mod):
    if hasattr(mod, 'weight_g'):
        return [mod.weight_g, mod.weight_v]
    return [mod.weight]


def apply_weight_norm(module, name='weight'):
    """Same parameters as torch.nn.utils.weight_norm(module, name, dim=0) -- weight_g
    (norm over all dims but 0) and weight_v -- without installing a forward hook: the
    effective weight is recomputed on the device by the HIP kernels at each use."""
    w = getattr(module, name)
    del module._parameters[name]
    with torch.no_grad():
        g = w.reshape(w.shape[0], -1).norm(dim=1).reshape([-1] + [1] * (w.dim() - 1))
    module.register_parameter(name + '_g', nn.Parameter(g.clone()))
    module.register_parameter(name + '_v', nn.Parameter(w.data.clone()))
    return module


class _ConvT:
    """conv_t's parameters as weight_of / weight_grad_to_params see them."""

    def __init__(self, ts):
        if len(ts) == 2:
            self.weight_g, self.weight_v = ts
        else:
            self.weight = ts[0]


def upsample_forward(x, params, k, wn, has_bias):
    """out[b, o, t*k + j] = sum_i x[b, i, t] W[i, o, j] + bias[o, j] as one GEMM (nn.py:33-43):
    (out, state for upsample_backward) -- srnn::upsample."""
    conv = _ConvT(params[:2] if wn else params[:1])
    bias_p = params[-1] if has_bias else None
    B, Cin, Lx = x.shape
    W = weight_of(conv)                                        # (Cin, Cout, k)
    Cout = W.shape[1]
    Wg = H.permute3(W, (2, 1, 0))                              # (k*Cout, Cin)
    xr = H.permute3(x.float(), (0, 2, 1)).reshape(B * Lx, Cin)  # (B*L, Cin)
    bias = None
    if bias_p is not None:
        bias = H.permute3(bias_p.reshape(1, Cout, k), (0, 2, 1)).reshape(-1)
    y = H.linear(xr, Wg.reshape(k * Cout, Cin), bias=bias)     # (B*L, k*Cout)
    out = H.permute3(y.reshape(B, Lx * k, Cout), (0, 2, 1))     # (B, Cout, L*k)
    st = _ConvT([None])
    st.conv, st.has_bias, st.xr, st.Wg = conv, has_bias, xr, Wg
    st.shape = (B, Cin, Lx, k, Cout)
    return out, st


def upsample_backward(st, dout):
    """(dx, [parameter gradients]) of upsample_forward -- srnn::upsample_bwd."""
    xr, Wg = st.xr, st.Wg
    B, Cin, Lx, k, Cout = st.shape
    dy = H.permute3(dout.float().contiguous(), (0, 2, 1)).reshape(B * Lx, k * Cout)
    dWg = H.gemm(dy, xr, transA=True)                          # (k*Cout, Cin)
    dx = H.gemm(dy, Wg.reshape(k * Cout, Cin))                 # (B*L, Cin)
    dx = H.permute3(dx.reshape(B, Lx, Cin), (0, 2, 1))
    dW = H.permute3(dWg.reshape(k, Cout, Cin), (2, 1, 0))      # (Cin, Cout, k)
    grads = weight_grad_to_params(st.conv, dW)
    if st.has_bias:
        db = H.colsum(dy, B * Lx, k * Cout)
        grads.append(H.permute3(db.reshape(1, k, Cout), (0, 2, 1)).reshape(Cout, k))
    return dx, grads


class LearnedUpsampling1d(nn.Module):
    """nn.py:7-43."""

    def __init__(self, in_channels, out_channels, kernel_size, bias=True):
        super().__init__()
        self.conv_t = nn.ConvTranspose1d(
            in_channels=in_channels, out_channels=out_channels, kernel_size=kernel_size,
            stride=kernel_size, bias=False)
        if bias:
            self.bias = nn.Parameter(torch.FloatTensor(out_channels, kernel_size))
        else:
            self.register_parameter('bias', None)
        self.reset_parameters()

    def reset_parameters(self):
        self.conv_t.reset_parameters()
        if self.bias is not None:
            nn.init.constant_(self.bias, 0)

    def forward(self, input):
        H.need_cuda(input)
        params = weight_params(self.conv_t) + ([self.bias] if self.bias is not None else [])
        import custom_ops
        out, _ = torch.ops.srnn.upsample(input, params, self.conv_t.kernel_size[0],
                                         hasattr(self.conv_t, 'weight_g'), self.bias is not None)
        return out


def lecun_uniform(tensor):
    """nn.py:46-48."""
    fan_in = nn.init._calculate_correct_fan(tensor, 'fan_in')
    nn.init.uniform_(tensor, -math.sqrt(3 / fan_in), math.sqrt(3 / fan_in))


def concat_init(tensor, inits):
    """nn.py:51-63."""
    try:
        tensor = tensor.data
    except AttributeError:
        pass
    (length, fan_out) = tensor.size()
    fan_in = length // len(inits)
    chunk = tensor.new(fan_in, fan_out)
    for (i, init) in enumerate(inits):
        init(chunk)
        tensor[i * fan_in: (i + 1) * fan_in, :] = chunk


# SRNN_FUSED_NLL=0 turns off the closed-form hand-over of the loss gradient to the MLP
# (custom_ops: srnn::nll_bits_bwd + srnn::mlp_bwd's nll_* arguments)
FUSED_NLL = os.environ.get('SRNN_FUSED_NLL', '1') != '0'


_NLL_ARGS = ('weight', 'size_average', 'ignore_index', 'reduce', 'reduction')


def _nll_options(args, kwargs):
    """nll_loss's optional arguments (weight, size_average, ignore_index, reduce, reduction),
    positional or keyword as the reference passes them through (nn.py:66-70) -> a dict."""
    if len(args) > len(_NLL_ARGS):
        raise TypeError('sequence_nll_loss_bits: too many positional arguments')
    opts = dict(zip(_NLL_ARGS, args))
    for k, v in kwargs.items():
        if k not in _NLL_ARGS:
            raise TypeError('sequence_nll_loss_bits: unexpected keyword argument %r' % k)
        if k in opts:
            raise TypeError('sequence_nll_loss_bits: got multiple values for %r' % k)
        opts[k] = v
    return opts


def sequence_nll_loss_bits(input, target, *args, **kwargs):
    """nn.py:66-70: NLL of log-probs (B, T, Q) x log2(e).  The reference's call (train.py:
    no extra arguments: the mean) runs on the HIP kernels (srnn::nll_bits); the optional
    nll_loss arguments are passed through as the reference does.  reduction='sum' is the HIP
    mean x rows; a class weight, an ignore_index that some target hits, or reduction='none'
    (none of which the reference's training uses) go to torch's nll_loss on the same device
    tensors."""
    H.need_cuda(input, target)
    import custom_ops
    if not (args or kwargs):
        return custom_ops.nll_bits(input, target)      # the registered op srnn::nll_bits
    opts = _nll_options(args, kwargs)
    size_average, reduce_ = opts.pop('size_average', None), opts.pop('reduce', None)
    if size_average is not None or reduce_ is not None:
        reduction = torch.nn.modules.loss._Reduction.legacy_get_string(size_average, reduce_)
    else:
        reduction = opts.get('reduction', 'mean')
    weight, ignore = opts.get('weight'), opts.get('ignore_index', -100)
    n_classes = input.size(2)
    # (targets are sample values in [0, Q): an ignore_index outside that never hits)
    hits_ignore = 0 <= ignore < n_classes and bool((target == ignore).any())
    if weight is None and not hits_ignore and reduction in ('mean', 'sum'):
        loss = custom_ops.nll_bits(input, target)
        return loss * target.numel() if reduction == 'sum' else loss
    return torch.nn.functional.nll_loss(
        input.reshape(-1, n_classes), target.reshape(-1), weight=weight, ignore_index=ignore,
        reduction=reduction) * math.log(math.e, 2)
