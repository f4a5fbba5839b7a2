"""Drop-in for the reference's optim.py (optim.py:1-21).

gradient_clipping(optimizer, min, max) returns the same wrapper: step(closure) runs the
closure, clamps every gradient to [min, max] in place (optim.py:11-13) and steps.  For
torch.optim.Adam over device parameters (train.py:238) the clamp and the Adam update
are ONE fused HIP kernel per parameter (srnn_adam_clip) operating on the optimizer's
own state tensors (step / exp_avg / exp_avg_sq), so Adam.state_dict() stays valid.
Parameters whose grad is None are treated as zero-grad, i.e. torch-0.4 zero_grad
semantics: the learned h0 keeps moving on its Adam moments on non-reset steps, as it
did in the reference's environment.  An optional `grad_sync` callable (set by
distributed.py) all-reduces gradients after the closure and before the clamp.
"""
import os

import torch

import samplernn_hip as H


class DeviceSteps:
    """Per-parameter-group count of completed Adam steps on the device (int64, one entry per
    group), read by srnn::adam_clip_ in place of a host step and advanced on the device by
    srnn::step_advance_ -- which skips while the persistent-sweep failure flag is up, as the
    update does.  A captured step (trainer graph mode) therefore replays with the right bias
    corrections.  `mirror[g]` is the value the host believes entry g holds (None: unknown);
    whenever it disagrees with the optimizer's own step count the entry is re-seeded."""

    def __init__(self, optimizer, device):
        self.t = torch.zeros(len(optimizer.param_groups), dtype=torch.int64, device=device)
        self.mirror = [0] * len(optimizer.param_groups)
        self.uniform = True       # every group's parameters share one step count


def _host_step(optimizer, group):
    for p in group['params']:
        st = optimizer.state.get(p)
        if st and 'step' in st:
            return int(st['step'].item())
    return None


def _advance_steps(items, optimizer=None, gi=0):
    """st['step'] += 1 for every (param, state) of a group, grouped by the new count.
    torch.optim keeps one 0-dim CPU step tensor per parameter (kept here for state_dict
    compatibility); a tensor op on each costs ~7 us of host time (0.5 ms per TBPTT step at 67
    parameters), so the step tensors are made views of ONE flat buffer (re-linked whenever a
    state dict was replaced, e.g. load_state_dict) and advanced by a single add."""
    if not items:
        return {}
    sts = [st for _, st in items]
    # the cache lives on the optimizer (it holds the group's state dicts)
    cache = optimizer.__dict__.setdefault('_srnn_step_bufs', {}) if optimizer is not None else {}
    e = cache.get(gi)
    if e is None or len(e[2]) != len(sts) or any(a is not b or a['step'] is not v
                                                 for a, b, v in zip(sts, e[2], e[1])):
        buf = torch.tensor([float(st['step']) for st in sts], dtype=torch.float32)
        views = [buf[i] for i in range(len(sts))]
        for st, v in zip(sts, views):
            st['step'] = v
        e = (buf, views, sts)
        cache[gi] = e
    e[0].add_(1.0)
    by_step = {}
    for it, v in zip(items, e[0].tolist()):
        by_step.setdefault(int(v), []).append(it)
    return by_step


def _fused_adam_step(optimizer, lo, hi, reduced=None, dsteps=None):
    """All parameters of a group that share a step count go through ONE multi-tensor
    launch (srnn_adam_clip_multi3) instead of one launch per tensor.  reduced: the data-
    parallel gradient buckets ((param, view) pairs, dtype, 1 / world scale; distributed.py)
    read in place instead of p.grad.  dsteps (DeviceSteps): take the step count from the
    device counters (re-seeded from the host count when they disagree) and advance them."""
    import custom_ops  # noqa: F401  (registers srnn::adam_clip_)
    zero = reduced is not None and reduced[0] == 'zero'
    if zero:
        # ZeRO-1 (distributed.GradAllReduce): this rank updates only its shard of each bucket;
        # pieces[id(p)] = [(a, b, gradient view)] -- elements [a, b) of p and their reduced sums
        import distributed as Dd
        pieces = {}
        for _, key, bucket, offs, s0, S, sh in reduced[1]:
            for i, a, b, so in Dd.zero_pieces([p.numel() for p in bucket], offs, s0, S):
                pieces.setdefault(id(bucket[i]), []).append((a, b, sh[so:so + b - a]))
        zero_shadows = []
        rv = None
        gscale = reduced[3]
    else:
        rv = {id(p): v for p, v in reduced[0]} if reduced else None
        gscale = reduced[2] if reduced else 1.0
    capturing = torch.cuda.is_current_stream_capturing()
    uniform = True
    for gi, group in enumerate(optimizer.param_groups):
        if group.get('weight_decay', 0) != 0 or group.get('amsgrad', False) or \
                group.get('maximize', False):
            raise NotImplementedError('fused clip+Adam: weight_decay/amsgrad/maximize')
        b1, b2 = group['betas']
        items = []
        for p in group['params']:
            if not p.requires_grad:
                continue
            st = optimizer.state[p]
            if len(st) == 0:
                st['step'] = torch.tensor(0.0, dtype=torch.float32)
                st['exp_avg'] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st['exp_avg_sq'] = torch.zeros_like(p, memory_format=torch.preserve_format)
            # a None grad goes to the kernel as NULL = all-zero (no zero-fill launch)
            if rv is None and not zero and p.grad is not None and (not p.grad.is_contiguous() or
                                                                   p.grad.dtype != torch.float32):
                p.grad = p.grad.float().contiguous()
            if not (p.is_contiguous() and p.dtype == torch.float32):
                raise NotImplementedError('fused clip+Adam: contiguous fp32 parameters only')
            items.append((p, st))
        by_step = _advance_steps(items, optimizer, gi)
        dstep = None
        if dsteps is not None and len(by_step) == 1:
            step = next(iter(by_step))
            if dsteps.mirror[gi] != step - 1:
                if capturing:
                    raise RuntimeError('fused Adam: device step counter out of step with the '
                                       'optimizer during graph capture')
                dsteps.t[gi].fill_(step - 1)
                dsteps.mirror[gi] = step - 1
            dstep = dsteps.t[gi:gi + 1]
        elif len(by_step) > 1:
            uniform = False
        for step, items in sorted(by_step.items()):
            # parameters with a cached bf16 copy (samplernn_hip.cast_param) get it rewritten
            # by the same kernel, so the next forward needs no cast
            shadows = [H.shadow_of(p) for p, _ in items]
            ev = H.roof_begin()
            nel = sum(p.numel() for p, _ in items)
            if zero:
                # the shard's pieces; every bf16 copy is refreshed after the parameter
                # all-gather (GradAllReduce.after_update), not here
                zero_shadows += [(p, sh) for (p, _), sh in zip(items, shadows) if sh is not None]
                pp, gg, mm, vv = [], [], [], []
                for p, s in items:
                    for a, b, gv in pieces.get(id(p), ()):
                        pp.append(p.view(-1)[a:b])
                        gg.append(gv)
                        mm.append(s['exp_avg'].view(-1)[a:b])
                        vv.append(s['exp_avg_sq'].view(-1)[a:b])
                torch.ops.srnn.adam_clip_(pp, gg, mm, vv, [None] * len(pp), float(gscale),
                                          float(lo), float(hi), float(group['lr']), float(b1),
                                          float(b2), float(group['eps']), step, dstep)
                H.roof_end('adam_clip', ev, sum(t.numel() for t in pp) * 32)
                continue
            grads = [p.grad for p, _ in items] if rv is None else [rv.get(id(p)) for p, _ in items]
            # the registered op srnn::adam_clip_ (custom_ops.py)
            torch.ops.srnn.adam_clip_([p for p, _ in items], grads,
                                      [s['exp_avg'] for _, s in items],
                                      [s['exp_avg_sq'] for _, s in items], shadows,
                                      float(gscale), float(lo), float(hi), float(group['lr']),
                                      float(b1), float(b2), float(group['eps']), step, dstep)
            for (p, _), sh in zip(items, shadows):
                if sh is not None:
                    H.shadow_refreshed(p)
            # algorithmic bytes: p, m, v read + written, the gradient read + written back
            # clamped (hardtanh_ in place, optim.py:13), the bf16 copies written
            H.roof_end('adam_clip', ev, nel * 32 + 2 * sum(
                p.numel() for (p, _), sh in zip(items, shadows) if sh is not None))
    if dsteps is not None:
        dsteps.uniform = uniform
        torch.ops.srnn.step_advance_(dsteps.t)
        dsteps.mirror = [None if m is None else m + 1 for m in dsteps.mirror]
    return zero_shadows if zero else None


def gradient_clipping(optimizer, min=-1, max=1, grad_sync=None):

    class OptimizerWrapper(object):

        def __init__(self):
            self.grad_sync = grad_sync
            self.dsteps = None        # DeviceSteps, created by the first fused step

        def _fused(self):
            return isinstance(optimizer, torch.optim.Adam) and all(
                p.is_cuda for g in optimizer.param_groups for p in g['params'])

        def zero_grad(self, set_to_none=None):
            """torch-0.4 semantics by default (zero-filled grads).  The fused step treats a
            None grad as zero, so there dropping the grads is equivalent and saves a fill
            per parameter plus the accumulate kernels of the next backward."""
            if set_to_none is None:
                set_to_none = self._fused()
            optimizer.zero_grad(set_to_none=set_to_none)

        def step(self, closure):
            if self._fused():
                if hasattr(self.grad_sync, 'zero_ok'):
                    self.grad_sync.zero_ok = True     # ZeRO-1 shards are read by this step
                with torch.enable_grad():
                    loss = closure()
                reduced = None
                if self.grad_sync is not None:
                    if hasattr(self.grad_sync, 'reduced'):      # distributed.GradAllReduce
                        self.grad_sync(optimizer, fused=True)
                        reduced = self.grad_sync.reduced
                    else:
                        self.grad_sync(optimizer)
                if self.dsteps is None or len(self.dsteps.mirror) != len(optimizer.param_groups):
                    # first step, or add_param_group since: one counter per group, re-seeded
                    # from the host step counts on this step
                    self.dsteps = DeviceSteps(optimizer, optimizer.param_groups[0]['params'][0].device)
                    self.dsteps.mirror = [None] * len(optimizer.param_groups)
                with torch.no_grad():
                    zs = _fused_adam_step(optimizer, min, max, reduced, self.dsteps)
                    if zs is not None:       # ZeRO-1: gather the updated shards
                        self.grad_sync.zero_shadows = zs
                        self.grad_sync.after_update()
                        self.grad_sync.zero_shadows = []
                return loss

            if hasattr(self.grad_sync, 'zero_ok'):
                self.grad_sync.zero_ok = False            # full reductions into p.grad

            def closure_wrapper():
                loss = closure()
                if self.grad_sync is not None:
                    self.grad_sync(optimizer)
                for group in optimizer.param_groups:
                    for p in group['params']:
                        if p.grad is None:
                            p.grad = torch.zeros_like(p)
                        p.grad.clamp_(min, max)
                return loss

            return optimizer.step(closure_wrapper)

        def rollback_steps(self, k):
            """Undo the Adam step-count increments of k steps whose update the device skipped
            (a persistent sweep gave up a hand-off, samplernn_hip.PersistentErrorWatch): the
            bias correction then matches the k fewer updates the moments hold."""
            for group in optimizer.param_groups:
                for p in group['params']:
                    st = optimizer.state.get(p)
                    if st and 'step' in st:
                        st['step'] -= k
            if self.dsteps is not None:        # re-seed the device counters on the next step
                self.dsteps.mirror = [None] * len(self.dsteps.mirror)

        # ---- graph mode (trainer/__init__.py): the step replayed from a captured graph
        def graph_ready(self):
            """True when the step can be captured: the fused path with device step counters
            whose groups each share one step count.  Under data parallelism the collectives
            are captured too (RCCL supports stream capture; tests/test_gpu_distributed.py
            test_graph_captured_dp_step_over_rccl) when the process group is 'nccl' -- gloo's
            host-side collectives cannot be -- unless SRNN_GRAPH_DP=0."""
            if not self._fused() or self.dsteps is None or not self.dsteps.uniform:
                return False
            if self.grad_sync is None:
                return True
            mode = os.environ.get('SRNN_GRAPH_DP', 'auto')
            if mode == '0':
                return False
            if mode == '1':
                return True
            import torch.distributed as dist
            return dist.is_available() and dist.is_initialized() and \
                dist.get_backend() == 'nccl'

        def graph_signature(self):
            """What a captured step baked in: hyper-parameters (kernel arguments) and the
            addresses of every parameter, moment and bf16 copy (kernel pointers)."""
            sig = []
            for group in optimizer.param_groups:
                sig.append((float(group['lr']), tuple(group['betas']), float(group['eps'])))
                for p in group['params']:
                    st = optimizer.state.get(p) or {}
                    sh = H.shadow_of(p)
                    sig.append((p.data_ptr(), st['exp_avg'].data_ptr() if 'exp_avg' in st else 0,
                                st['exp_avg_sq'].data_ptr() if 'exp_avg_sq' in st else 0,
                                sh.data_ptr() if sh is not None else 0))
            return tuple(sig)

        def before_replay(self):
            """Re-seed any device counter that disagrees with the optimizer's step count."""
            for gi, group in enumerate(optimizer.param_groups):
                step = _host_step(optimizer, group)
                if step is not None and self.dsteps.mirror[gi] != step:
                    self.dsteps.t[gi].fill_(step)
                    self.dsteps.mirror[gi] = step

        def after_replay(self):
            """The host bookkeeping the replayed step did not run: step counts + 1."""
            for gi, group in enumerate(optimizer.param_groups):
                # the same item list _fused_adam_step advances (requires_grad AND state), so
                # the flat step buffer is reused and a frozen parameter's count stays put
                _advance_steps([(p, st) for p in group['params'] if p.requires_grad
                                for st in (optimizer.state.get(p),) if st and 'step' in st],
                               optimizer, gi)
            self.dsteps.mirror = [None if m is None else m + 1 for m in self.dsteps.mirror]

        def __getattr__(self, attr):
            return getattr(optimizer, attr)

    return OptimizerWrapper()
