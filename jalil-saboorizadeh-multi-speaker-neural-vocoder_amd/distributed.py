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
  * the loss is a mean over equal shards, so the mean of rank losses is the global loss.

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
    SRNN_DIST_BACKEND overrides (e.g. gloo for a rehearsal on one GPU)."""
    if world() <= 1 or (dist.is_available() and dist.is_initialized()):
        return
    if backend is None:
        backend = os.environ.get('SRNN_DIST_BACKEND') or \
            ('nccl' if torch.cuda.device_count() > 0 else 'gloo')
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    if backend == 'nccl':
        torch.cuda.set_device(device_index())
        dist.init_process_group(backend, device_id=torch.device('cuda', device_index()))
    else:
        dist.init_process_group(backend)


def shard_rows(total_rows, r=None, n=None):
    """Contiguous stream-row range owned by rank r."""
    r = rank() if r is None else r
    n = world() if n is None else n
    if total_rows % n:
        raise ValueError('global batch %d not divisible by world size %d' % (total_rows, n))
    per = total_rows // n
    return slice(r * per, (r + 1) * per)


class GradAllReduce:
    """Average gradients across ranks in flat buckets of ~bucket_mb, in place.

    Used as `gradient_clipping(..., grad_sync=GradAllReduce())`: runs after the closure's
    backward and before the clamp + Adam.  Parameters without a grad contribute zeros
    (torch-0.4 zero_grad semantics), so every rank reduces identical bucket layouts.
    """

    def __init__(self, bucket_mb=64, group=None):
        self.bucket_bytes = int(bucket_mb * (1 << 20))
        self.group = group
        self._bufs = {}

    def __call__(self, optimizer):
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
            return
        n = dist.get_world_size(self.group)
        params = [p for g in optimizer.param_groups for p in g['params'] if p.requires_grad]
        for p in params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        buckets, cur, size = [], [], 0
        for p in params:
            nb = p.numel() * p.grad.element_size()
            if cur and size + nb > self.bucket_bytes:
                buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += nb
        if cur:
            buckets.append(cur)
        for bi, bucket in enumerate(buckets):
            total = sum(p.numel() for p in bucket)
            key = (bi, total, bucket[0].grad.dtype, bucket[0].grad.device)
            flat = self._bufs.get(key)
            if flat is None:
                flat = torch.empty(total, dtype=bucket[0].grad.dtype, device=bucket[0].grad.device)
                self._bufs[key] = flat
            off = 0
            for p in bucket:
                k = p.numel()
                flat[off:off + k].copy_(p.grad.reshape(-1))
                off += k
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
            flat.mul_(1.0 / n)
            off = 0
            for p in bucket:
                k = p.numel()
                p.grad.copy_(flat[off:off + k].view_as(p.grad))
                off += k


def barrier():
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def max_over_ranks(x, device=None):
    """Max of a python float over ranks (used for the timed region)."""
    if not (dist.is_available() and dist.is_initialized()):
        return x
    t = torch.tensor([float(x)], dtype=torch.float64,
                     device=device if device is not None else 'cpu')
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
