"""CPU ORACLE -- test infrastructure, NOT product code.

A from-scratch fp32 restatement, in plain PyTorch CPU ops, of the reference's hot
path (mahdeslami11/jalil-saboorizadeh-Multi-speaker-Neural-Vocoder @ /root/reference):
the conditional SampleRNN forward (Predictor), the autoregressive Generator loop, the
NLL-in-bits loss and the clipped-Adam TBPTT step.  Every function cites the reference
file:line it restates.

Only tests/, __graft_entry__.smoke() and bench.py's `cpu_baseline` leg may import
this module, and only as the CHECKER / the timed CPU baseline ("kind": "port").
The product path (the HIP library behind the drop-in model.py) never routes here.

Parity of this oracle is PINNED against golden vectors produced by running the
reference itself in the survey container (tests/golden/make_golden.py; tests in
tests/test_oracle_golden.py).
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

LOG2E = math.log(math.e, 2)          # nn.py:70
MU = 255.0                            # utils.py:29
LOG_MU1 = 5.5451774444795623          # utils.py:30
EPSILON = 1e-2                        # utils.py:6
EPSILONs = 1e-6                       # utils.py:45


# ----------------------------------------------------------------- µ-law (utils.py)
def ulaw(x, max_value=1.0):
    """utils.py:33-36."""
    v = MU / max_value
    return x.sign() * (v * x.abs() + 1.).log() / LOG_MU1


def iulaw(c):
    """utils.py:39-42."""
    x = (c.abs() * LOG_MU1).exp() - 1
    return c.sign() * x / MU


def midrise(x, q_levels=256):
    """utils.py:48-51 (truncation toward zero of the scaled value)."""
    x = 0.5 * (x + 1.0)
    x = x * (q_levels - EPSILONs)
    return x.long()


def imidrise(xq, q_levels=256):
    """utils.py:54-55."""
    return xq.float() * 2.0 / q_levels - 1.0


def uquantize(samples, q_levels):
    """utils.py:58-59."""
    return midrise(ulaw(samples), q_levels)


def udequantize(samples, q_levels):
    """utils.py:62-63."""
    return iulaw(imidrise(samples, q_levels))


def linear_quantize(samples, q_levels):
    """utils.py:9-15 (1-D rows)."""
    s = samples.clone()
    s -= s.min(dim=-1)[0]
    s /= s.max(dim=-1)[0]
    s *= q_levels - EPSILON
    s += EPSILON / 2
    return s.long()


def linear_dequantize(samples, q_levels):
    """utils.py:18-19."""
    return samples.float() / (q_levels / 2) - 1


def q_zero(q_levels):
    """utils.py:22-23."""
    return q_levels // 2


# ----------------------------------------------------------------- model
def cumprod(xs):
    out, p = [], 1
    for x in xs:
        p *= int(x)
        out.append(p)
    return out


def weight_norm_w(g, v):
    """torch weight_norm(dim=0): w = g * v / ||v|| over all dims but 0 (model.py:119-131,177-178,303-306)."""
    n = v.reshape(v.shape[0], -1).norm(dim=1)
    return v * (g.reshape(-1) / n).reshape([-1] + [1] * (v.dim() - 1))


class OracleSampleRNN:
    """Functional restatement of SampleRNN / FrameLevelRNN / SampleLevelMLP (model.py:18-325).

    `params` maps reference state_dict names (Predictor prefix 'model.') to fp32 tensors.
    """

    def __init__(self, frame_sizes, n_rnn, dim, q_levels, weight_norm, cond_dim, spk_dim,
                 params):
        self.frame_sizes = list(frame_sizes)
        self.n_rnn = n_rnn
        self.dim = dim
        self.q_levels = q_levels
        self.weight_norm = weight_norm
        self.cond_dim = cond_dim
        self.spk_dim = spk_dim
        self.nfs = cumprod(frame_sizes)
        self.p = params
        self.hidden = [None] * len(frame_sizes)   # Runner.hidden_states (model.py:335-336)

    @property
    def lookback(self):
        """model.py:60-62."""
        return self.nfs[-1]

    # -- parameter helpers
    def _w(self, prefix):
        if (prefix + '.weight') in self.p:
            return self.p[prefix + '.weight']
        return weight_norm_w(self.p[prefix + '.weight_g'], self.p[prefix + '.weight_v'])

    def tier(self, k, prev, upper, cond, spk, h):
        """FrameLevelRNN.forward (model.py:180-263).

        prev (B,F,nfs) fp32, upper (B,F,D) or None, cond (B,F,C), spk (B,1) int,
        h (n_rnn,B,D) or None -> (out (B,F*fs,D), h_new (n_rnn,B,D)).
        """
        P = 'model.frame_level_rnns.%d.' % k
        B, Fr, _ = prev.shape
        D = self.dim
        x = F.linear(prev, self._w(P + 'input_expand')[:, :, 0], self.p[P + 'input_expand.bias'])
        if upper is not None:                                  # model.py:199-200
            x = x + upper
        else:                                                  # model.py:202-218
            c = F.linear(cond.float(), self._w(P + 'cond_expand')[:, :, 0],
                         self.p[P + 'cond_expand.bias'])
            x = x + c
            e = self.p[P + 'spk_embedding.weight'][spk.long()]           # (B,1,S)
            s = F.linear(e.float(), self._w(P + 'spk_expand')[:, :, 0],
                         self.p[P + 'spk_expand.bias'])                 # (B,1,D)
            x = x + s
        if h is None:                                          # model.py:224-228
            h = self.p[P + 'h0'].unsqueeze(1).expand(self.n_rnn, B, D)
        # torch.nn.GRU (model.py:148-153, 244): the same fused ATen GRU the reference's module
        # runs (gate order r | z | n: n = tanh(W_in x + b_in + r (W_hn h + b_hn)),
        # h' = (1 - z) n + z h), called functionally on the state_dict tensors
        flat = []
        for l in range(self.n_rnn):
            flat += [self.p[P + 'rnn.weight_ih_l%d' % l], self.p[P + 'rnn.weight_hh_l%d' % l],
                     self.p[P + 'rnn.bias_ih_l%d' % l], self.p[P + 'rnn.bias_hh_l%d' % l]]
        layer_in, h_new = torch._VF.gru(x, h.contiguous(), flat, True, self.n_rnn, 0.0,
                                        torch.is_grad_enabled(), False, True)
        # LearnedUpsampling1d (nn.py:33-43): out[b,t*k+j,o] = sum_i y[b,t,i] W[i,o,j] + bias[o,j]
        W = weight_norm_w(self.p[P + 'upsampling.conv_t.weight_g'],
                          self.p[P + 'upsampling.conv_t.weight_v'])
        fs = self.frame_sizes[k]
        out = F.conv_transpose1d(layer_in.permute(0, 2, 1), W, stride=fs)  # (B,D,F*fs)
        out = out + self.p[P + 'upsampling.bias'].unsqueeze(0).unsqueeze(2).expand(
            B, D, Fr, fs).reshape(B, D, Fr * fs)
        return out.permute(0, 2, 1), h_new

    def mlp(self, x, upper):
        """SampleLevelMLP.forward (model.py:308-325): x (B,T+FS0-1) int, upper (B,T,D) -> logp (B,T,Q)."""
        P = 'model.sample_level_mlp.'
        B = upper.shape[0]
        Q = self.q_levels
        e = self.p[P + 'embedding.weight'][x.reshape(-1)].reshape(B, -1, Q).permute(0, 2, 1)
        a = F.relu(F.conv1d(e, self._w(P + 'input')) + upper.permute(0, 2, 1))
        a = F.relu(F.conv1d(a, self._w(P + 'hidden'), self.p[P + 'hidden.bias']))
        z = F.conv1d(a, self._w(P + 'output'), self.p[P + 'output.bias']).permute(0, 2, 1)
        return F.log_softmax(z.reshape(-1, Q), dim=1).reshape(B, -1, Q)

    def reset_hidden_states(self):
        self.hidden = [None] * len(self.frame_sizes)

    def predict(self, inp, reset, cond, spk):
        """Predictor.forward (model.py:357-436) incl. TBPTT hidden carry + detach (model.py:348)."""
        if reset:
            self.reset_hidden_states()
        B = inp.shape[0]
        L = self.lookback
        upper = None
        for k in reversed(range(len(self.frame_sizes))):
            n = self.nfs[k]
            prev = 2 * udequantize(inp[:, L - n: -n + 1], self.q_levels)
            prev = prev.reshape(B, -1, n)
            if upper is None:
                upper, h = self.tier(k, prev, None, cond.reshape(B, -1, cond.shape[-1]),
                                     spk.reshape(B, -1), self.hidden[k])
            else:
                upper, h = self.tier(k, prev, upper, None, None, self.hidden[k])
            self.hidden[k] = h.detach()
        fs0 = self.frame_sizes[0]
        return self.mlp(inp[:, L - fs0:], upper)

    @torch.no_grad()
    def generate(self, n_seqs, cond, spk, noise, return_logp=False):
        """Generator.__call__ (model.py:445-520) with sampling written as argmax(p/q).

        cond: (N,C) shared by all rows (reference) or (n_seqs,N,C) per row; spk: int or (n_seqs,).
        noise: (T, n_seqs, Q) Exp(1) draws, q_t consumed at step t exactly as
        `multinomial(1)` does in torch>=2 CPU (p/q then argmax, first max); None: drawn from
        torch's CPU generator step by step, as the reference's multinomial does.
        Returns int64 sequences (n_seqs, L+T) (and logp (n_seqs,T,Q) if asked).
        """
        cond = torch.as_tensor(np.asarray(cond))
        if cond.dim() == 2:
            cond = cond.unsqueeze(0).expand(n_seqs, *cond.shape)
        spk = torch.as_tensor(np.asarray(spk)).reshape(-1).long()
        if spk.numel() == 1:
            spk = spk.expand(n_seqs)
        spk = spk.reshape(n_seqs, 1)
        N = cond.shape[1]
        L = self.lookback
        T = N * L                                           # model.py:455 (seq_len ignored)
        Q = self.q_levels
        seq = torch.full((n_seqs, L + T), q_zero(Q), dtype=torch.long)  # model.py:459
        self.reset_hidden_states()
        outs = [None] * len(self.frame_sizes)
        logps = []
        fs0 = self.frame_sizes[0]
        for i in range(L, L + T):                           # model.py:462
            for k in reversed(range(len(self.frame_sizes))):
                n = self.nfs[k]
                if i % n != 0:
                    continue
                prev = 2 * udequantize(seq[:, i - n: i], Q).unsqueeze(1)   # model.py:470-476
                if k == len(self.frame_sizes) - 1:
                    j = i // L - 1                          # model.py:483
                    out, h = self.tier(k, prev, None, cond[:, j:j + 1], spk, self.hidden[k])
                else:
                    fi = (i // n) % self.frame_sizes[k + 1]  # model.py:491-495
                    out, h = self.tier(k, prev, outs[k + 1][:, fi:fi + 1], None, None,
                                       self.hidden[k])
                self.hidden[k] = h
                outs[k] = out
            upper = outs[0][:, i % fs0: i % fs0 + 1]         # model.py:511-513
            lp = self.mlp(seq[:, i - fs0: i], upper)[:, 0]   # model.py:504-516
            p = lp.exp()
            q = noise[i - L] if noise is not None else torch.empty(n_seqs, Q).exponential_(1)
            seq[:, i] = torch.argmax(p / q, dim=-1)             # model.py:517 (multinomial)
            if return_logp:
                logps.append(lp)
        if return_logp:
            return seq, torch.stack(logps, 1)
        return seq


def sequence_nll_loss_bits(logp, target):
    """nn.py:66-70: mean NLL x log2(e)."""
    Q = logp.shape[-1]
    return F.nll_loss(logp.reshape(-1, Q), target.reshape(-1)) * LOG2E


class OracleAdam:
    """optim.py:4-21 gradient_clipping(-1,1) + torch.optim.Adam (train.py:238), torch-2.10
    single-tensor update order, torch-0.4 zero_grad (grads zero-filled, never None)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        self.params = params
        self.lr, self.b1, self.b2, self.eps = lr, betas[0], betas[1], eps
        self.m = [torch.zeros_like(p) for p in params]
        self.v = [torch.zeros_like(p) for p in params]
        self.step_n = 0

    @torch.no_grad()
    def step(self, grads):
        self.step_n += 1
        bc1 = 1 - self.b1 ** self.step_n
        bc2 = 1 - self.b2 ** self.step_n
        step_size = self.lr / bc1
        bc2s = bc2 ** 0.5
        for p, g, m, v in zip(self.params, grads, self.m, self.v):
            g = g.clamp(-1.0, 1.0)                              # optim.py:13 hardtanh_
            m.lerp_(g, 1 - self.b1)
            v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            denom = (v.sqrt() / bc2s).add_(self.eps)
            p.addcdiv_(m, denom, value=-step_size)


def tbptt_step(model, opt, names, batch, return_grads=True):
    """Trainer.train body (trainer/__init__.py:62-117): forward, loss, backward, clip, Adam.

    Returns (loss float, clipped grads list -- None without return_grads: the timed CPU
    baseline does not pay for a copy the reference step does not make)."""
    inp, reset, tgt, cond, spk = batch
    params = [model.p[n] for n in names]
    for p in params:
        p.requires_grad_(True)
        p.grad = None
    logp = model.predict(inp, reset, cond, spk)
    loss = sequence_nll_loss_bits(logp, tgt)
    loss.backward()
    grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in params]
    clipped = [g.clamp(-1, 1) for g in grads] if return_grads else None
    opt.step(grads)
    for p in params:
        p.grad = None
    return float(loss.detach()), clipped


def from_state_dict(cfg, sd):
    params = {k: torch.as_tensor(np.asarray(v)).float().clone() for k, v in sd.items()}
    return OracleSampleRNN(cfg['frame_sizes'], cfg['n_rnn'], cfg['dim'], cfg['q_levels'],
                           cfg['weight_norm'], cfg['cond_dim'], cfg['spk_dim'], params)
