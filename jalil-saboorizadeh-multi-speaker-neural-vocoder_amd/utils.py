"""Drop-in for the reference's utils.py (utils.py:1-63): mu-law / linear quantisers.

Same names, signatures and results.  Device tensors run the HIP kernels of
libsamplernn_hip.so; host tensors (the DataLoader side, dataset.py:253-254) run the
library's host quantiser built from the same reference-pinned tables, so both are
bit-exact to the reference for every float32/float64 input in [-1, 1].
"""
import torch

import samplernn_hip as H

EPSILON = 1e-2
MU = 255.
LOG_MU1 = 5.5451774444795623    # log(1+MU)
EPSILONs = 1e-6


def linear_quantize(samples, q_levels):
    """utils.py:9-15 (host-side data preparation; not on the device hot path)."""
    samples = samples.clone()
    samples -= samples.min(dim=-1)[0].expand_as(samples)
    samples /= samples.max(dim=-1)[0].expand_as(samples)
    samples *= q_levels - EPSILON
    samples += EPSILON / 2
    return samples.long()


def linear_dequantize(samples, q_levels):
    """utils.py:18-19."""
    if samples.is_cuda:
        return _dequant(samples, q_levels, 1.0, mode=1)
    return samples.float() / (q_levels / 2) - 1


def q_zero(q_levels):
    """utils.py:22-23."""
    return q_levels // 2


def ulaw(x, max_value=1.0):
    """utils.py:33-36 (elementwise helper kept for API completeness)."""
    v = MU / max_value
    return x.sign() * (v * x.abs() + 1.).log() / LOG_MU1


def iulaw(c, max_value=1.0, mu=255.):
    """utils.py:39-42."""
    x = (c.abs() * LOG_MU1).exp() - 1
    return c.sign() * x / MU


def midrise(x, q_levels=256):
    """utils.py:48-51."""
    x = 0.5 * (x + 1.0)
    x *= (q_levels - EPSILONs)
    return x.long()


def imidrise(xq, q_levels=256):
    """utils.py:54-55."""
    return xq.float() * 2.0 / q_levels - 1.0


def uquantize(samples, q_levels):
    """utils.py:58-59: midrise(ulaw(x)) -> int64 indices (bit-exact)."""
    if samples.dtype not in (torch.float32, torch.float64):
        samples = samples.float()
    x = samples.contiguous()
    out = torch.empty(x.shape, dtype=torch.long, device=x.device)
    n = x.numel()
    if x.is_cuda:
        name = 'srnn_uquantize_f64' if x.dtype == torch.float64 else 'srnn_uquantize_f32'
        H.lib().call(name, H.ptr(x), H.ptr(out), n, q_levels, H.stream())
    else:
        name = 'srnn_uquantize_f64_host' if x.dtype == torch.float64 else 'srnn_uquantize_f32_host'
        H.lib().call(name, H.ptr(x), H.ptr(out), n, q_levels)
    return out


def _dequant(samples, q_levels, scale, mode=0):
    """scale * dequantize(samples) on the device: the registered op srnn::dequant."""
    import custom_ops  # noqa: F401  (registers the op)
    with torch.no_grad():           # (integer input: no gradient; keeps outputs grad-free)
        return torch.ops.srnn.dequant(samples, q_levels, float(scale), mode)


def _dequant_impl(samples, q_levels, scale, mode=0):
    if samples.is_cuda and samples.dtype == torch.long and samples.dim() == 2 and \
            samples.stride(1) == 1 and not samples.is_contiguous():
        # a window of the index stream: read in place (no copy of the slice first)
        out = torch.empty(samples.shape, dtype=torch.float32, device=samples.device)
        H.lib().call('srnn_udequantize2d', H.ptr(samples), samples.stride(0), H.ptr(out),
                     samples.shape[0], samples.shape[1], q_levels, scale, mode, H.stream())
        return out
    k = samples.long().contiguous()
    out = torch.empty(k.shape, dtype=torch.float32, device=k.device)
    H.lib().call('srnn_udequantize', H.ptr(k), H.ptr(out), k.numel(), q_levels, scale, mode,
                 H.stream())
    return out


def udequantize(samples, q_levels):
    """utils.py:62-63: iulaw(imidrise(k)) (bit-exact LUT for q_levels = 256)."""
    if samples.is_cuda:
        return _dequant(samples, q_levels, 1.0, mode=0)
    k = samples.long().contiguous()
    out = torch.empty(k.shape, dtype=torch.float32)
    H.lib().call('srnn_udequantize_host', H.ptr(k), H.ptr(out), k.numel(), q_levels)
    return out
