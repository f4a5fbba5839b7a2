"""Data-parallel TBPTT over one node: one process per GPU, RCCL over xGMI.

The reference has no distributed code; this is the MI355X-native addition
for the TBPTT step:

  * rows, not items, are sharded: the stateful TBPTT layout (dataset.py:155-163) makes
    row b of every chunk a continuation of the same stream, so rank r owns stream rows
    [r*B/N, (r+1)*B/N) for every chunk and its GRU hidden states never move;
  * one exchange per step: gradients are averaged with bucketed all-reduces
    (torch.distributed 'nccl' = RCCL on ROCm) AFTER backward and BEFORE the [-1, 1]
    clamp, so the clamp sees the full-batch gradient exactly as the reference's
    single-process step does (optim.py:11-13);
  * the loss is a mean over equal shards, so the mean of rank losses is the global loss;
  * a persistent GRU sweep that gave up a hand-off raises a device flag (persist.hip); the
    flag rides in the last gradient bucket, so every rank's fused clip+Adam skips the step
    and every rank's Trainer raises, together (no rank is left waiting in a collective).

Generation needs no collective: utterances are independent (replicas only).
"""
import os

import torch
import torch.distributed as dist


def world():
    return int(os.environ.get('WORLD_SIZE', '1'))


def rank():
    return int(os.environ.get('RANK', '0'))


def local_rank():
    return int(os.environ.get('LOCAL_RANK', '0'))


def device_index():
    """GPU of this rank: LOCAL_RANK (modulo the visible devices, so a multi-rank rehearsal
    can share one GPU with the gloo backend)."""
    n = torch.cuda.device_count()
    return local_rank() % n if n > 0 else 0


def init(backend=None):
    """Initialise the process group from torchrun's env (no-op for a single process).
    Backend: 'nccl' (= RCCL on ROCm) when GPUs are present, else 'gloo';
    SRNN_DIST_BACKEND overrides (e.g. gloo for a rehearsal on one GPU); SRNN_DP_FORCE=1 also
    builds a one-rank group (the DP step's collectives measured on a one-GPU box)."""
    if (world() <= 1 and os.environ.get('SRNN_DP_FORCE', '0') != '1') or \
            (dist.is_available() and dist.is_initialized()):
        return
    if backend is None:
        backend = os.environ.get('SRNN_DIST_BACKEND') or \
            ('nccl' if torch.cuda.device_count() > 0 else 'gloo')
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    for k, v in (('RANK', '0'), ('WORLD_SIZE', '1'), ('MASTER_PORT', '29533')):
        os.environ.setdefault(k, v)             # a forced one-rank group outside torchrun
    if backend == 'nccl':
        torch.cuda.set_device(device_index())
        dist.init_process_group(backend, device_id=torch.device('cuda', device_index()))
    else:
        dist.init_process_group(backend)
    _declare_device_share()


def device_key():
    """(host, PCI address, UUID) of this rank's GPU: the physical device, whatever
    HIP/ROCR/CUDA_VISIBLE_DEVICES renumbering each process sees."""
    import socket
    p = torch.cuda.get_device_properties(device_index())
    return (socket.gethostname(), '%04x:%02x:%02x' % (p.pci_domain_id, p.pci_bus_id,
                                                      p.pci_device_id), str(p.uuid))


def device_share(keys, mine):
    """How many ranks' device keys name this rank's physical GPU."""
    return sum(1 for k in keys if tuple(k) == tuple(mine))


def _declare_device_share():
    """Ranks that map onto one physical GPU (a rehearsal: two ranks on one card) each run
    persistent sweeps on it at once.  Their grids are only co-resident if they fit the device
    together, so the HIP library is told how many processes share it
    (samplernn_hip.set_device_share): launches are then sized to 1/share of the CUs or take
    the per-step kernels -- declared up front instead of a sweep waiting on CUs that another
    process's sweep holds.  The share is counted from the real device mapping: every rank's
    (host, PCI address, UUID) is all-gathered once at init and this rank counts the ranks
    naming its own card -- correct for per-rank *_VISIBLE_DEVICES isolation (each process
    sees one device 0), for launchers that set no LOCAL_WORLD_SIZE (srun / mpirun) and for
    several nodes.  SRNN_DEVICE_SHARE overrides."""
    n = torch.cuda.device_count()
    if n <= 0:
        return 1
    env = os.environ.get('SRNN_DEVICE_SHARE')
    if env:
        share = max(1, int(env))
    elif dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        mine = device_key()
        keys = [None] * dist.get_world_size()
        dist.all_gather_object(keys, mine)
        share = device_share(keys, mine)
    else:
        share = 1
    if share > 1:
        import warnings
        import samplernn_hip as H
        warnings.warn('%d ranks share each GPU: persistent kernels are sized to 1/%d of its CUs'
                      % (share, share))
        H.set_device_share(share)
    return share


def shard_rows(total_rows, r=None, n=None):
    """Contiguous stream-row range owned by rank r."""
    r = rank() if r is None else r
    n = world() if n is None else n
    if total_rows % n:
        raise ValueError('global batch %d not divisible by world size %d' % (total_rows, n))
    per = total_rows // n
    return slice(r * per, (r + 1) * per)


def readiness_groups(model):
    """Parameters of a SampleRNN (or Predictor) in the order backward produces their grads:
    the sample-level MLP first, then the tiers bottom -> top; the learned h0 rows last (they
    only get a gradient on reset chunks, so they must not hold a bucket back)."""
    m = getattr(model, 'model', model)
    groups = [[p for p in m.sample_level_mlp.parameters() if p.requires_grad]]
    h0 = []
    for rnn in m.frame_level_rnns:
        ps = []
        for name, p in rnn.named_parameters():
            if not p.requires_grad:
                continue
            (h0 if name == 'h0' else ps).append(p)
        groups.append(ps)
    groups.append(h0)
    return [g for g in groups if g]


_ALIGN = 64          # bucket offsets in elements (16-B aligned views for the fused Adam)


def _grad_dtype(name):
    name = (name or os.environ.get('SRNN_DP_GRAD_DTYPE', 'fp32')).lower()
    if name in ('fp32', 'float32'):
        return torch.float32
    if name in ('bf16', 'bfloat16'):
        return torch.bfloat16
    raise ValueError('gradient bucket dtype %r (fp32 / bf16)' % name)


class GradAllReduce:
    """Average gradients across ranks in flat buckets of ~bucket_mb, before the clamp.

    Used as `gradient_clipping(..., grad_sync=GradAllReduce())`: runs after the closure's
    backward and before the clamp + Adam.  Parameters without a grad contribute zeros
    (torch-0.4 zero_grad semantics), so every rank reduces identical bucket layouts.

    Device path (the fused clip+Adam, optim.py): a bucket is packed by ONE multi-tensor launch
    (srnn_pack_grads: every gradient of the bucket into the flat buffer at 64-element-aligned
    offsets, converted to the bucket dtype) and SUM-reduced in place; the fused Adam then
    reads the reduced bucket through views with a 1 / world scale (srnn_adam_clip_multi2) --
    no per-parameter copy launches, no unpack, no separate mean pass, and the local gradients
    are released once packed.  grad_dtype 'bf16' (or env SRNN_DP_GRAD_DTYPE=bf16) halves the
    bytes on xGMI: each rank's gradient is rounded to bf16 before the reduction (the sum of
    N bf16 terms accumulates in bf16 inside RCCL); the default fp32 keeps the reference's
    full-batch gradient to fp32 rounding.  Host path (CPU / non-fused optimizers): the same
    buckets, unpacked into p.grad.

    overlap_groups (e.g. readiness_groups(model)): parameter groups in the order backward
    completes them.  A post-accumulate-grad hook packs a group's bucket and starts its
    all-reduce asynchronously (RCCL on its own stream, ordered after the producing kernels)
    as soon as the group's last gradient lands, so the MLP's and the bottom tier's
    reductions run under the rest of the backward; __call__ then only waits.  Groups whose
    grads never arrive this step (h0 on non-reset chunks) are reduced at the sync point.
    A persistent GRU sweep enqueued while reductions are in flight first makes the stream
    wait for them (_fence): RCCL kernels and a sweep never share the CUs.  So that the fence
    does not hold a sweep behind a large bucket that became ready just before it (the bottom
    tier's 92 MB in front of the top tier's reverse sweep), a ready bucket is launched only
    once the next persistent sweep has been enqueued (_after_sweep, samplernn_hip
    AFTER_PERSISTENT) -- its pack and RCCL kernels are then ordered after that sweep and run
    under the GEMMs that follow it -- or at the sync point at the latest (defer=False, or
    env SRNN_DP_DEFER=0, launches at once).  close() removes the hooks and the fence.
    """

    def __init__(self, bucket_mb=64, group=None, overlap_groups=None, grad_dtype=None,
                 defer=None, zero=None, force=None):
        self.bucket_bytes = int(bucket_mb * (1 << 20))
        # ZeRO-1 (fused device path only): reduce-scatter the buckets, clamp + Adam on this
        # rank's shard, all-gather the parameters (see _zero_* below).  Opt-in (SRNN_DP_ZERO=1):
        # it saves (N - 1) / N of the clip + Adam pass (0.22 ms per step) but the all-gather of
        # every parameter after the update cannot overlap the backward like the all-reduce's
        # buckets do
        self.zero = os.environ.get('SRNN_DP_ZERO', '0') == '1' if zero is None else bool(zero)
        # force: run the bucket path even in a one-rank group (tests of the collectives and
        # their graph capture on a one-GPU box); SRNN_DP_FORCE=1
        self.force = os.environ.get('SRNN_DP_FORCE', '0') == '1' if force is None else force
        self._zplan = None          # ZeRO: key -> (bucket, offs, total, shard) of the fused path
        self._pflat = {}            # ZeRO: key -> flat fp32 parameter buffer (params are views)
        self._gshard = {}           # ZeRO: key -> this rank's reduced gradient shard
        self.zero_shadows = []      # ZeRO: (param, bf16 copy) pairs the fused step left stale
        self.zero_ok = False        # set by optim.gradient_clipping when its step is the fused one
        self.defer = os.environ.get('SRNN_DP_DEFER', '1') != '0' if defer is None else defer
        self._deferred = []         # ready buckets waiting for the next sweep's enqueue
        self._after_ref = None
        self.group = group
        self.grad_dtype = _grad_dtype(grad_dtype)
        self._bufs = {}
        self._groups = None
        self._hooks = []
        self._pending = {}
        self._fenced = set()
        self._flag_buf = None
        self._fence_ref = None
        self.reduced = None         # fused path: ([(param, view)], dtype, scale) of the step
        if overlap_groups is not None and dist.is_available() and dist.is_initialized() and \
                (dist.get_world_size(group) > 1 or self.force):
            self._install(overlap_groups)

    # ---- bucketing
    def _split(self, params):
        buckets, cur, size = [], [], 0
        es = torch.tensor([], dtype=self.grad_dtype).element_size()
        for p in params:
            nb = p.numel() * es
            if cur and size + nb > self.bucket_bytes:
                buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += nb
        if cur:
            buckets.append(cur)
        return buckets

    def _offsets(self, bucket):
        offs, off = [], 0
        for p in bucket:
            offs.append(off)
            off += (p.numel() + _ALIGN - 1) // _ALIGN * _ALIGN
        if self._zero_on(bucket):
            # equal 64-element-aligned shards (the pieces of a parameter a shard holds then
            # start 256-B aligned for the fused Adam's vector accesses)
            q = _ALIGN * self._n()
            off = (off + q - 1) // q * q
        return offs, off

    def _n(self):
        return dist.get_world_size(self.group)

    def _zero_on(self, bucket):
        # only under the fused device clip + Adam (optim.gradient_clipping sets zero_ok), which
        # reads the shards; any other optimizer gets fully reduced gradients in p.grad
        return self.zero and self.zero_ok and bucket[0].is_cuda

    def _flat(self, key, bucket, flag):
        offs, total = self._offsets(bucket)
        dev = bucket[0].device
        dtype = self.grad_dtype if dev.type == 'cuda' else torch.float32
        k = (key, flag, total, dtype, dev)
        flat = self._bufs.get(k)
        if flat is None:
            flat = torch.empty(total + (_ALIGN if flag else 0), dtype=dtype, device=dev)
            self._bufs[k] = flat
        return flat, offs, total

    def _launch(self, key, bucket, async_op, flag=False):
        """Pack a bucket and start its SUM all-reduce.  flag: the bucket carries one extra
        element, this rank's persistent-sweep failure flag (0 / 1, persist.hip), so after the
        reduction every rank holds the same verdict."""
        flat, offs, total = self._flat(key, bucket, flag)
        if flat.is_cuda:
            import ctypes
            import samplernn_hip as H
            n = len(bucket)
            srcs = []
            for p in bucket:
                g = p.grad
                if g is not None and (g.dtype != torch.float32 or not g.is_contiguous()):
                    g = g.float().contiguous()
                    p.grad = g
                srcs.append(g)
            H.lib().call('srnn_pack_grads', n,
                         (ctypes.c_void_p * n)(*[H.ptr(g) for g in srcs]),
                         (ctypes.c_int64 * n)(*[p.numel() for p in bucket]),
                         (ctypes.c_int64 * n)(*offs), H.ptr(flat), H.dcode(flat), H.stream())
            if flag:
                _flag_to(flat[total:total + 1])
        else:
            flat.zero_()
            for p, o in zip(bucket, offs):
                if p.grad is not None:
                    flat[o:o + p.numel()].copy_(p.grad.reshape(-1))
        if self._zero_on(bucket):
            # ZeRO-1: this rank receives only the SUM of its shard
            S = total // self._n()
            sh = self._gshard.get(key)
            if sh is None or sh.numel() != S or sh.dtype != flat.dtype:
                sh = torch.empty(S, dtype=flat.dtype, device=flat.device)
                self._gshard[key] = sh
            if dist.get_backend(self.group) == 'nccl':
                work = dist.reduce_scatter_tensor(sh, flat[:total], op=dist.ReduceOp.SUM,
                                                  group=self.group, async_op=async_op)
            else:        # gloo has no reduce-scatter: reduce everything, keep the shard
                work = dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group,
                                       async_op=async_op)
            return (flat, offs, total, key), work
        work = dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group, async_op=async_op)
        return (flat, offs, total, key), work

    def _finish(self, bucket, rec, n, fused, views):
        flat, offs, total, key = rec
        if flat.numel() > total:        # the carried failure flag: any rank's -> this rank's
            _flag_from(flat[total:total + 1])
        if fused and self._zero_on(bucket):
            S = total // n
            r = dist.get_rank(self.group)
            sh = self._gshard[key]
            if dist.get_backend(self.group) != 'nccl':
                sh.copy_(flat[r * S:(r + 1) * S])
            self._zero_params(key, bucket, offs, total)
            views.append(('zero', key, bucket, offs, r * S, S, sh))
            for p in bucket:
                p.grad = None           # the local gradient was packed: release it
            return
        if fused:
            for p, o in zip(bucket, offs):
                views.append((p, flat[o:o + p.numel()].view(p.shape)))
                p.grad = None           # the local gradient was packed: release it
            return
        flat.mul_(1.0 / n)
        for p, o in zip(bucket, offs):
            v = flat[o:o + p.numel()].view(p.shape)
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            p.grad.copy_(v)

    # ---- overlapped mode
    def _install(self, groups):
        import weakref
        import samplernn_hip as H
        ref = weakref.WeakMethod(self._fence)
        self._fence_ref = ref
        H.BEFORE_PERSISTENT.append(ref)
        self._after_ref = weakref.WeakMethod(self._after_sweep)
        H.AFTER_PERSISTENT.append(self._after_ref)
        self._groups = []
        for gi, params in enumerate(groups):
            for bi, bucket in enumerate(self._split(params)):
                self._groups.append(((gi, bi), bucket))
        self._owner = {}
        for idx, (_, bucket) in enumerate(self._groups):
            for p in bucket:
                self._owner[id(p)] = idx
        self._ready = [0] * len(self._groups)
        # the hooks hold this object weakly: parameters outlive a GradAllReduce that is dropped
        me = weakref.ref(self)

        def hook(p):
            s = me()
            if s is not None:
                s._on_grad(p)
        for idx, (_, bucket) in enumerate(self._groups):
            for p in bucket:
                self._hooks.append(p.register_post_accumulate_grad_hook(hook))

    def close(self):
        """Remove the gradient hooks and the persistent-sweep fence (and drop the buckets)."""
        for h in self._hooks:
            h.remove()
        self._hooks = []
        if self._fence_ref is not None:
            import samplernn_hip as H
            H.BEFORE_PERSISTENT[:] = [f for f in H.BEFORE_PERSISTENT if f is not self._fence_ref]
            H.AFTER_PERSISTENT[:] = [f for f in H.AFTER_PERSISTENT if f is not self._after_ref]
            self._fence_ref = self._after_ref = None
        self._bufs = {}
        self._groups = None

    def _fence(self):
        """Before a persistent GRU sweep: the current stream waits for every all-reduce in
        flight (a stream-level wait under RCCL, no host synchronisation), so the sweep never
        shares the CUs with RCCL kernels (samplernn_hip.BEFORE_PERSISTENT)."""
        for idx, (rec, work) in self._pending.items():
            if idx not in self._fenced:
                work.wait()
                self._fenced.add(idx)

    def _on_grad(self, p):
        idx = self._owner[id(p)]
        self._ready[idx] += 1
        key, bucket = self._groups[idx]
        if self._ready[idx] == len(bucket) and idx not in self._pending and \
                idx not in self._deferred:
            if self.defer:
                self._deferred.append(idx)
            else:
                self._pending[idx] = self._launch(key, bucket, True)

    def _launch_deferred(self):
        for idx in self._deferred:
            key, bucket = self._groups[idx]
            self._pending[idx] = self._launch(key, bucket, True)
        self._deferred = []

    def _after_sweep(self):
        """Right after a persistent sweep is enqueued: start the buckets that became ready
        before it (ordered after it on the stream)."""
        self._launch_deferred()

    def __call__(self, optimizer, fused=False):
        """Reduce this step's gradients.  fused=True (the device clip+Adam): leave them in the
        buckets and publish (param, view) pairs, the dtype and the 1 / world scale in
        self.reduced; otherwise write the means back into p.grad."""
        self.reduced = None
        if not (dist.is_available() and dist.is_initialized()) or \
                (dist.get_world_size() == 1 and not self.force):
            return
        n = dist.get_world_size(self.group)
        views = []
        if self._groups is not None:
            # every backward kernel is enqueued by now, so the failure flag read here covers
            # all persistent sweeps of the step: it rides in the last bucket launched here, or
            # alone when the hooks already launched every bucket (reset chunks)
            late = [idx for idx in range(len(self._groups)) if idx not in self._pending]
            self._deferred = []                       # (launched below, in index order)
            dev = self._groups[0][1][0].is_cuda
            zero = self._zero_on(self._groups[0][1])
            for idx in late:                          # grads that never arrived this step
                key, bucket = self._groups[idx]
                self._pending[idx] = self._launch(key, bucket, True,
                                                  flag=dev and not zero and idx == late[-1])
            solo = None
            if dev and (zero or not late):
                # (ZeRO: a shard holds 1/N of a bucket, so the flag travels on its own)
                if self._flag_buf is None:
                    self._flag_buf = torch.zeros(1, device=self._groups[0][1][0].device)
                _flag_to(self._flag_buf)
                solo = dist.all_reduce(self._flag_buf, op=dist.ReduceOp.SUM, group=self.group,
                                       async_op=True)
            for idx, (key, bucket) in enumerate(self._groups):
                rec, work = self._pending[idx]
                work.wait()
                self._finish(bucket, rec, n, fused and dev, views)
            if solo is not None:
                solo.wait()
                _flag_from(self._flag_buf)
            self._pending = {}
            self._fenced = set()
            self._ready = [0] * len(self._groups)
        else:
            params = [p for g in optimizer.param_groups for p in g['params'] if p.requires_grad]
            buckets = self._split(params)
            zero = bool(buckets) and self._zero_on(buckets[0]) and fused
            if zero:
                if self._flag_buf is None:
                    self._flag_buf = torch.zeros(1, device=buckets[0][0].device)
                _flag_to(self._flag_buf)
                dist.all_reduce(self._flag_buf, op=dist.ReduceOp.SUM, group=self.group)
                _flag_from(self._flag_buf)
            for bi, bucket in enumerate(buckets):
                dev = bucket[0].is_cuda
                rec, _ = self._launch(bi, bucket, False,
                                      flag=dev and not zero and bi == len(buckets) - 1)
                self._finish(bucket, rec, n, fused and dev, views)
        if views and views[0][0] == 'zero':
            self.reduced = ('zero', views, views[0][6].dtype, 1.0 / n)
        elif views:
            self.reduced = (views, views[0][1].dtype, 1.0 / n)


    # ---- ZeRO-1 (reduce-scatter -> sharded clamp + Adam -> all-gather; the same
    # bytes on xGMI as the all-reduce, 1/N of the optimizer's HBM traffic per rank).  The
    # clamp is elementwise (optim.py:11-13) and Adam is elementwise too, so updating each
    # rank's shard of the SUMMED gradient (scaled by 1/N) and gathering the parameters gives
    # every rank exactly the replicated update.
    def _zero_params(self, key, bucket, offs, total):
        """Parameters of a ZeRO bucket become views of one flat fp32 buffer (once), so the
        all-gather writes them in place."""
        pf = self._pflat.get(key)
        if pf is not None and all(p.data_ptr() == pf[o:].data_ptr()
                                  for p, o in zip(bucket, offs)):
            return
        pf = torch.zeros(total, dtype=torch.float32, device=bucket[0].device)
        with torch.no_grad():
            for p, o in zip(bucket, offs):
                if p.dtype != torch.float32 or not p.is_contiguous():
                    raise NotImplementedError('ZeRO-1: contiguous fp32 parameters only')
                v = pf[o:o + p.numel()]
                v.copy_(p.data.reshape(-1))
                p.data = v.view(p.shape)
        self._pflat[key] = pf

    def after_update(self):
        """After the fused clamp + Adam updated this rank's shards (ZeRO-1): all-gather every
        bucket's parameters in place, then refresh the parameters' bf16 copies.  The current
        stream waits for the gathers (a stream-level wait: the next forward is ordered after
        them without a host synchronisation)."""
        red = self.reduced
        if red is None or red[0] != 'zero':
            return
        import ctypes
        import samplernn_hip as H
        n = self._n()
        nccl = dist.get_backend(self.group) == 'nccl'
        works = []
        for _, key, bucket, offs, s0, S, _sh in red[1]:
            pf = self._pflat[key]
            if nccl:
                works.append(dist.all_gather_into_tensor(pf, pf[s0:s0 + S], group=self.group,
                                                         async_op=True))
            else:
                parts = list(pf.split(S))
                dist.all_gather(parts, pf[s0:s0 + S].clone(), group=self.group)
        for w in works:
            w.wait()
        src, dst, cnt, ps = [], [], [], []
        for p, sh in self.zero_shadows:
            src.append(H.ptr(p))
            dst.append(H.ptr(sh))
            cnt.append(p.numel())
            ps.append(p)
        if src:
            k = len(src)
            H.lib().call('srnn_cast_multi', k, (ctypes.c_void_p * k)(*src),
                         (ctypes.c_void_p * k)(*dst), (ctypes.c_int64 * k)(*cnt), H.stream())
            for p in ps:
                H.shadow_refreshed(p)


def zero_pieces(numels, offs, s0, S):
    """ZeRO-1 shard map of one bucket: the parameters at flat offsets `offs` (numels
    elements each) intersected with this rank's shard [s0, s0 + S) of the flat index space ->
    [(parameter index, first element, end element, offset into the shard)].  Every element
    of every parameter lies in exactly one rank's shard (tests/test_distributed_cpu.py)."""
    out = []
    for i, (n, o) in enumerate(zip(numels, offs)):
        a, b = max(o, s0), min(o + n, s0 + S)
        if b > a:
            out.append((i, a - o, b - o, a - s0))
    return out


def _flag_to(dst):
    """dst (1-element fp32 / bf16 device tensor) = this rank's persistent-sweep failure flag."""
    import samplernn_hip as H
    H.lib().call('srnn_persistent_flag_to', H.ptr(dst), H.dcode(dst), H.stream())


def _flag_from(src):
    """Raise this rank's failure flag if the reduced value says any rank failed: the fused
    clip+Adam then skips the update on every rank and every rank's Trainer raises."""
    import samplernn_hip as H
    H.lib().call('srnn_persistent_flag_or', H.ptr(src), H.dcode(src), H.stream())


def gather_rows(local, total_rows):
    """Concatenate every rank's contiguous row shard (host tensor (rows, ...)) in rank order;
    identity for one process.  Over the process group's backend: RCCL (device tensors) under
    nccl, the host under gloo."""
    if not _active():
        return local
    dev = _coll_device()
    t = local.to(dev).contiguous()
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    out = torch.cat(parts, 0).cpu()
    assert out.shape[0] == total_rows
    return out


def barrier():
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def _active():
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def _coll_device():
    """Where a small host-value collective runs: the rank's GPU under nccl (RCCL reduces
    device tensors only), the CPU under gloo."""
    if dist.get_backend() == 'nccl':
        return torch.device('cuda', torch.cuda.current_device())
    return torch.device('cpu')


def sum_over_ranks(values):
    """Element-wise sum of a list of python floats over ranks (identity for one process)."""
    if not _active():
        return [float(v) for v in values]
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=_coll_device())
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(v) for v in t.tolist()]


def mean_over_ranks(x):
    """Mean of a python float over ranks: the global loss of a row-sharded step (every rank
    holds an equal shard, so the mean of shard means is the full-batch mean)."""
    if not _active():
        return float(x)
    return sum_over_ranks([x])[0] / dist.get_world_size()


def max_over_ranks(x, device=None):
    """Max of a python float over ranks (used for the timed region)."""
    if not (dist.is_available() and dist.is_initialized()):
        return x
    t = torch.tensor([float(x)], dtype=torch.float64,
                     device=device if device is not None else 'cpu')
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
