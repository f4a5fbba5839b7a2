"""world_size-2 gloo tests of the data-parallel TBPTT layer (distributed.py) on CPU.

The HIP model needs a GPU, so the DP mechanics are exercised with a CPU stand-in
recurrent model: rank r owns stream rows shard_rows(B, r, 2), gradients are averaged
by GradAllReduce before the [-1, 1] clamp, and the result must equal a single-process
full-batch step."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Toy(torch.nn.Module):
    """Row-independent recurrent stand-in: h_t = tanh(W x_t + U h_{t-1}), loss = mean."""

    def __init__(self):
        super().__init__()
        g = torch.Generator().manual_seed(0)
        self.W = torch.nn.Parameter(torch.randn(5, 3, generator=g))
        self.U = torch.nn.Parameter(torch.randn(5, 5, generator=g) * 0.3)
        self.h0 = torch.nn.Parameter(torch.zeros(5))

    def forward(self, x, h):
        import samplernn_hip as H
        B, T, _ = x.shape
        if h is None:
            h = self.h0.expand(B, 5)
        out = []
        for t in range(T):
            h = torch.tanh(x[:, t] @ self.W.t() + h @ self.U.t())
            if t == T // 2:
                # stands in for a persistent GRU sweep inside the backward: the fence makes
                # it wait for every all-reduce already in flight (results must not change)
                h.register_hook(lambda g: (H.before_persistent_sweep(),
                                           H.after_persistent_sweep(), g)[2])
            out.append(h)
        return torch.stack(out, 1), h.detach()


def _data(B=8, T=6, chunks=3):
    g = torch.Generator().manual_seed(1)
    return torch.randn(chunks, B, T, 3, generator=g) * 3


def _train(model, data, rows, grad_sync):
    import optim
    opt = optim.gradient_clipping(torch.optim.SGD(model.parameters(), lr=0.1), -1, 1,
                                  grad_sync=grad_sync)
    h = None
    losses = []
    for n in range(data.shape[0]):
        x = data[n][rows]

        def closure():
            nonlocal h
            out, h_new = model(x, h if n > 0 else None)
            loss = (out ** 2).mean() * 40.0          # large grads so the clamp is active
            loss.backward()
            closure.h = h_new
            return loss
        opt.zero_grad(set_to_none=False)
        losses.append(float(opt.step(closure).detach()))
        h = closure.h
    return losses, [p.detach().clone() for p in model.parameters()]


def _worker(rank, world, port, q, overlap=False, defer=True):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import distributed as D
    D.init(backend='gloo')
    data = _data()
    rows = D.shard_rows(data.shape[1])
    model = _Toy()
    # overlapped mode: hooks start each group's all-reduce when its last grad lands; h0 in
    # its own group (it has no grad on non-reset chunks in the real model)
    groups = [[model.U], [model.W], [model.h0]] if overlap else None
    losses, params = _train(model, data, rows,
                            D.GradAllReduce(bucket_mb=0.0001, overlap_groups=groups,
                                            defer=defer))
    loss_t = torch.tensor(losses)
    dist.all_reduce(loss_t)
    if rank == 0:
        q.put(((loss_t / world).tolist(), [p.tolist() for p in params]))
    dist.destroy_process_group()


@pytest.mark.parametrize('overlap,defer', [(False, True), (True, True), (True, False)])
def test_dp_two_ranks_equals_full_batch(overlap, defer):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, overlap, defer))
             for r in range(2)]
    for p in procs:
        p.start()
    losses_dp, params_dp = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    losses, params = _train(_Toy(), _data(), slice(0, 8), None)
    assert torch.allclose(torch.tensor(losses_dp), torch.tensor(losses), atol=1e-5)
    for a, b in zip(params_dp, params):
        assert torch.allclose(torch.tensor(a), b, atol=1e-5)


def test_shard_rows():
    import distributed as D
    assert D.shard_rows(512, 3, 8) == slice(192, 256)
    with pytest.raises(ValueError):
        D.shard_rows(10, 0, 3)


class _FakeTrainer:
    cuda = False

    def __init__(self, shift):
        self.shift = shift
        self.stats = {}

    def model(self, inputs, reset, cond, spk, writer, idx):
        return inputs.float() + self.shift

    @staticmethod
    def criterion(out, target):
        return (out - target.float()).abs().mean()


def _plugin_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import distributed as D
    from trainer.plugins import TrainingLossMonitor, ValidationPlugin
    D.init(backend='gloo')
    # rank r sees rows r*2 .. r*2+1 of a 4-row batch; per-rank losses differ
    full = torch.arange(4 * 3, dtype=torch.float32).reshape(4, 3)
    rows = D.shard_rows(4)
    batch = [(full[rows], torch.ones(1), torch.zeros(2, 3), torch.zeros(2, 1), torch.zeros(2, 1))]
    tr = _FakeTrainer(shift=0.0)
    vp = ValidationPlugin(batch, batch, None)
    vp.register(tr)
    val = vp._evaluate(batch, 0)
    mon = TrainingLossMonitor()
    mon.register(tr)
    local = float(full[rows].mean())
    mon.iteration(1, None, None, None, torch.tensor(local))
    q.put((rank, val, tr.stats['training_loss']['last']))
    dist.destroy_process_group()


def test_dp_plugins_report_full_batch_losses():
    """Under DP the validation loss and the logged training loss are the full-batch values,
    not rank 0's shard (ValidationPlugin sums (loss, rows), TrainingLossMonitor averages)."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_plugin_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = torch.arange(12, dtype=torch.float32).reshape(4, 3).mean().item()
    for _, val, tl in got:
        assert abs(val - full) < 1e-9
        assert abs(tl - full) < 1e-6


class _Work:
    def __init__(self):
        self.waits = 0

    def wait(self):
        self.waits += 1


def test_fence_waits_every_pending_reduction_and_unregisters():
    """GradAllReduce._fence (registered in samplernn_hip.BEFORE_PERSISTENT through a weak
    reference) makes a persistent sweep wait for EVERY all-reduce in flight, once each; close()
    and garbage collection both take it off the list (no stale fences or buckets pile up)."""
    import gc
    import distributed as D
    import samplernn_hip as H
    before = list(H.BEFORE_PERSISTENT)
    sync = D.GradAllReduce(bucket_mb=1)
    sync._install([[torch.nn.Parameter(torch.zeros(3))], [torch.nn.Parameter(torch.zeros(2))]])
    assert len(H.BEFORE_PERSISTENT) == len(before) + 1
    w = [_Work(), _Work(), _Work()]
    sync._pending = {0: (None, w[0]), 1: (None, w[1])}
    H.before_persistent_sweep()
    assert [x.waits for x in w] == [1, 1, 0]
    sync._pending[2] = (None, w[2])
    H.before_persistent_sweep()                  # only the newly launched one is waited for
    assert [x.waits for x in w] == [1, 1, 1]
    sync.close()
    assert H.BEFORE_PERSISTENT == before
    sync2 = D.GradAllReduce(bucket_mb=1)
    sync2._install([[torch.nn.Parameter(torch.zeros(3))]])
    assert len(H.BEFORE_PERSISTENT) == len(before) + 1
    del sync2
    gc.collect()
    H.before_persistent_sweep()                  # the dead entry is dropped
    assert H.BEFORE_PERSISTENT == before


def test_bucket_offsets_aligned():
    import distributed as D
    ps = [torch.nn.Parameter(torch.zeros(n)) for n in (3, 64, 65, 1)]
    offs, total = D.GradAllReduce(zero=False)._offsets(ps)
    assert offs == [0, 64, 128, 256] and total == 320


def test_ready_buckets_wait_for_the_next_sweep():
    """defer (default): a bucket whose gradients are complete is launched right after the next
    persistent sweep is enqueued (samplernn_hip.AFTER_PERSISTENT), so the sweep's fence never
    waits for it; the sync point launches whatever is still deferred, in index order."""
    import distributed as D
    import samplernn_hip as H
    a, b = torch.nn.Parameter(torch.zeros(3)), torch.nn.Parameter(torch.zeros(2))
    sync = D.GradAllReduce(bucket_mb=1, defer=True)
    sync._install([[a], [b]])
    launched = []
    sync._launch = lambda key, bucket, async_op, flag=False: (launched.append(key),
                                                             (None, _Work()))[1]
    sync._on_grad(a)
    assert launched == [] and sync._deferred == [0]
    H.before_persistent_sweep()                  # nothing in flight: nothing to wait for
    H.after_persistent_sweep()                   # the sweep is enqueued: bucket 0 goes
    assert launched == [(0, 0)] and 0 in sync._pending and sync._deferred == []
    sync._on_grad(b)
    assert launched == [(0, 0)] and sync._deferred == [1]
    sync.close()
    assert sync._after_ref is None


@pytest.mark.parametrize('world', [1, 2, 3, 8])
def test_zero_shards_cover_every_element_once(world):
    """ZeRO-1's shard map (distributed.zero_pieces over GradAllReduce's 64-aligned, world-padded
    bucket layout): across the ranks every element of every parameter is updated exactly once,
    pieces start 64-element aligned (16-B vector access in the fused Adam), and each piece's
    gradient offset points at the same flat element."""
    import distributed as D
    sizes = [3, 64, 65, 1, 1000, 4096, 7]
    ps = [torch.nn.Parameter(torch.zeros(n)) for n in sizes]
    # the bucket layout GradAllReduce._offsets builds for a ZeRO bucket: 64-aligned offsets,
    # total padded to a multiple of 64 x world (the padding step needs device parameters
    # there, so it is restated here)
    offs, raw = D.GradAllReduce(zero=False)._offsets(ps)
    q = 64 * world
    total = (raw + q - 1) // q * q
    assert total % (64 * world) == 0
    S = total // world
    seen = [torch.zeros(n, dtype=torch.int32) for n in sizes]
    for r in range(world):
        for i, a, b, so in D.zero_pieces(sizes, offs, r * S, S):
            assert a % 64 == 0 or a == 0
            assert offs[i] + a == r * S + so          # gradient view = the same flat element
            seen[i][a:b] += 1
    assert all(bool((x == 1).all()) for x in seen)


class _Sync:
    group = None


class _Opt:
    grad_sync = _Sync()


def _agree_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import distributed as D
    from trainer import _capture_agreed
    D.init(backend='gloo')
    both_ok = _capture_agreed(_Opt(), True)
    one_failed = _capture_agreed(_Opt(), rank != 1)
    q.put((rank, both_ok, one_failed))
    dist.destroy_process_group()


def test_graph_capture_outcome_agreed_across_ranks():
    """Trainer._capture under data parallelism: the ranks agree on the capture's outcome
    (MIN all-reduce), so a capture failing on one rank sends EVERY rank back to the eager
    step -- no rank replays captured collectives while another issues them eagerly (ADVICE
    r04).  Without a process group the local outcome stands."""
    from trainer import _capture_agreed
    assert _capture_agreed(_Opt(), True) is True and _capture_agreed(_Opt(), False) is False
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_agree_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(got) == [(0, True, False), (1, True, False)]
