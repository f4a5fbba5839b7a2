"""Data-parallel TBPTT with the real HIP model, world size 2 on one GPU.

The driver's 8-GPU runs use RCCL; a one-GPU box cannot host two RCCL ranks, so this
rehearsal runs both ranks on cuda:0 with the gloo backend (distributed.device_index maps
LOCAL_RANK onto the visible devices).  What it covers that test_distributed_cpu's toy
model does not: GradAllReduce's overlap hooks on the HIP autograd outputs (_TierFn /
MLP), the late h0 group (grads only on reset chunks), the failure flag riding in the last
bucket, the fused clip+Adam with NULL gradients, and the Trainer loop — checked against
the reference's own full-batch trajectory (tests/golden/tbptt_t3.npz: B = 2, so each rank
owns one stream row).  Tolerances as test_gpu_parity.test_tbptt_golden.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, name, overlap, zero, q):
    try:
        sys.path[:0] = [HERE, os.path.join(HERE, 'golden'),
                        os.path.join(os.path.dirname(HERE),
                                     'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd')]
        os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
        import distributed as D
        import nn as snn
        import optim
        import recipe
        import samplernn_hip as H
        from conftest import golden
        from test_gpu_parity import build
        from trainer import Trainer
        D.init(backend='gloo')
        H.lib()
        if zero == 'nccl_emul':
            D.dist = _NcclEmul(D.dist)
            zero = True
        g = golden('tbptt_' + name)
        cfg = recipe.CONFIGS[name]
        m, pred = build(cfg, recipe.make_weights(cfg, int(g['weight_seed'])))
        B = int(g['B'])
        rows = D.shard_rows(B)
        sync = D.GradAllReduce(bucket_mb=0.01, zero=zero,
                               overlap_groups=D.readiness_groups(pred) if overlap else None)
        opt = optim.gradient_clipping(torch.optim.Adam(pred.parameters(), lr=float(g['lr'])),
                                      grad_sync=sync)
        losses = []

        def criterion(out, tgt):
            loss = snn.sequence_nll_loss_bits(out, tgt)
            losses.append(float(loss.detach()))
            return loss
        data = [(torch.from_numpy(g['input_%d' % s])[rows],
                 torch.tensor([int(g['reset_%d' % s])] * (rows.stop - rows.start)),
                 torch.from_numpy(g['target_%d' % s])[rows],
                 torch.from_numpy(g['cond_%d' % s])[rows],
                 torch.from_numpy(g['spk_%d' % s])[rows])
                for s in range(int(g['n_steps']))]
        tr = Trainer(pred, criterion, opt, data, True, None)
        tr.run(1)
        torch.cuda.synchronize()
        H.check_persistent_errors()
        glob = [D.mean_over_ranks(x) for x in losses]
        params = {k: p.detach().cpu().numpy().copy() for k, p in pred.named_parameters()}
        q.put((rank, glob, params, None))
        D.barrier()
        import torch.distributed as dist
        dist.destroy_process_group()
    except Exception as e:          # surface the failure instead of a queue timeout
        import traceback
        q.put((rank, None, None, traceback.format_exc()))
        raise


class _Done:
    def wait(self):
        return True


class _NcclEmul:
    """torch.distributed as distributed.py sees it under RCCL, on a gloo group: get_backend
    says 'nccl', so GradAllReduce takes its RCCL-only ZeRO branches (reduce_scatter_tensor into
    the shard, the in-place all_gather_into_tensor of the flat parameters), and those two
    collectives are restated with their documented semantics over gloo's all_reduce /
    all_gather -- the shard offsets of the RCCL form are then checked against the reference's
    full-batch trajectory without two GPUs."""

    def __init__(self, real):
        self._d = real

    def __getattr__(self, k):
        return getattr(self._d, k)

    def get_backend(self, group=None):
        return 'nccl'

    def reduce_scatter_tensor(self, out, inp, op=None, group=None, async_op=False):
        tmp = inp.clone()
        self._d.all_reduce(tmp, op=self._d.ReduceOp.SUM, group=group)
        r, S = self._d.get_rank(group), out.numel()
        out.copy_(tmp[r * S:(r + 1) * S])
        return _Done() if async_op else None

    def all_gather_into_tensor(self, out, inp, group=None, async_op=False):
        parts = list(out.split(inp.numel()))
        self._d.all_gather(parts, inp.clone(), group=group)
        return _Done() if async_op else None


@pytest.mark.parametrize('overlap,zero', [(True, True), (False, True), (True, False),
                                          (False, False), (True, 'nccl_emul'),
                                          (False, 'nccl_emul')])
def test_dp_two_ranks_match_reference_full_batch(hip, overlap, zero):
    """zero: ZeRO-1 (each rank clamps + updates its shard of the summed gradient, then the
    parameters are all-gathered) or the replicated update after an all-reduce; 'nccl_emul'
    runs ZeRO-1's RCCL branches over gloo (_NcclEmul)."""
    from conftest import golden
    name = 't3'
    g = golden('tbptt_' + name)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, name, overlap, zero, q))
             for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(2):
        rank, losses, params, err = q.get(timeout=100)
        assert err is None, 'rank %d failed:\n%s' % (rank, err)
        got[rank] = (losses, params)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    names = [str(s) for s in g['names']]
    for rank in (0, 1):
        losses, params = got[rank]
        np.testing.assert_allclose(losses, g['losses'], atol=1e-4, rtol=0)
        for k in names:
            np.testing.assert_allclose(params[k], g['param_final/' + k], atol=2e-4, rtol=0,
                                       err_msg='rank %d %s' % (rank, k))
    # both ranks hold the same replica after every step
    for k in names:
        np.testing.assert_array_equal(got[0][1][k], got[1][1][k], err_msg=k)


def _flag_worker(rank, world, port, overlap, dtype, zero, q):
    """Rank 0 raises its persistent-sweep failure flag before a step: the flag rides in the
    last gradient bucket, so BOTH ranks' fused clip+Adam skip the update (weights and moments
    unchanged) and both ranks' checks raise (distributed.py, persist.hip)."""
    try:
        sys.path[:0] = [HERE, os.path.join(HERE, 'golden'),
                        os.path.join(os.path.dirname(HERE),
                                     'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd')]
        os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
        import distributed as D
        import nn as snn
        import optim
        import recipe
        import samplernn_hip as H
        from conftest import golden
        from test_gpu_parity import build
        D.init(backend='gloo')
        H.lib()
        g = golden('tbptt_t3')
        cfg = recipe.CONFIGS['t3']
        m, pred = build(cfg, recipe.make_weights(cfg, int(g['weight_seed'])))
        rows = D.shard_rows(int(g['B']))
        sync = D.GradAllReduce(bucket_mb=0.01, grad_dtype=dtype, zero=zero,
                               overlap_groups=D.readiness_groups(pred) if overlap else None)
        opt = optim.gradient_clipping(torch.optim.Adam(pred.parameters(), lr=1e-3),
                                      grad_sync=sync)
        dev = 'cuda'

        def step(s):
            inp = torch.from_numpy(g['input_%d' % s])[rows].to(dev)
            tgt = torch.from_numpy(g['target_%d' % s])[rows].to(dev)
            cond = torch.from_numpy(g['cond_%d' % s])[rows].to(dev)
            spk = torch.from_numpy(g['spk_%d' % s])[rows].to(dev)
            opt.zero_grad()

            def closure():
                loss = snn.sequence_nll_loss_bits(pred(inp, True, cond, spk), tgt)
                loss.backward()
                return loss
            return opt.step(closure)
        step(0)
        H.check_persistent_errors()
        before = [p.detach().clone() for p in pred.parameters()] + \
                 [opt.state[p]['exp_avg'].clone() for p in pred.parameters()]
        if rank == 0:
            one = torch.ones(1, device=dev)
            H.lib().call('srnn_persistent_flag_or_f32', H.ptr(one), H.stream())
        step(1)
        torch.cuda.synchronize()
        after = [p.detach().clone() for p in pred.parameters()] + \
                [opt.state[p]['exp_avg'].clone() for p in pred.parameters()]
        unchanged = all(torch.equal(a, b) for a, b in zip(before, after))
        raised = False
        try:
            H.check_persistent_errors()
        except RuntimeError:
            raised = True
        q.put((rank, unchanged, raised, None))
        sync.close()
        D.barrier()
        import torch.distributed as dist
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, None, None, traceback.format_exc()))
        raise


def _spawn(target, extra, world=2, timeout=150):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port) + extra + (q,))
             for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        item = q.get(timeout=timeout)
        assert item[-1] is None, 'rank %d failed:\n%s' % (item[0], item[-1])
        got[item[0]] = item[1:-1]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    return got


@pytest.mark.parametrize('overlap', [True, False])
@pytest.mark.parametrize('dtype', ['fp32', 'bf16'])
@pytest.mark.parametrize('zero', [True, False])
def test_dp_failure_flag_skips_every_rank(hip, overlap, dtype, zero):
    got = _spawn(_flag_worker, (overlap, dtype, zero))
    for rank in (0, 1):
        unchanged, raised = got[rank]
        assert unchanged, 'rank %d moved its weights / moments on a failed step' % rank
        assert raised, 'rank %d did not raise' % rank


def _bf16_bucket_worker(rank, world, port, q):
    """The reference's 3-step TBPTT trajectory with bf16 gradient buckets (each rank's gradient
    rounded to bf16 before the SUM): losses and final parameters stay within bf16-communication
    tolerance of the reference's full-batch fp32 trajectory."""
    try:
        os.environ['SRNN_DP_GRAD_DTYPE'] = 'bf16'
        _worker(rank, world, port, 't3', True, True, q)
    except Exception:
        raise


def test_dp_bf16_buckets_track_reference(hip):
    from conftest import golden
    g = golden('tbptt_t3')
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bf16_bucket_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(2):
        rank, losses, params, err = q.get(timeout=100)
        assert err is None, 'rank %d failed:\n%s' % (rank, err)
        got[rank] = (losses, params)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    names = [str(s) for s in g['names']]
    for rank in (0, 1):
        losses, params = got[rank]
        np.testing.assert_allclose(losses, g['losses'], atol=2e-3, rtol=0)
        worst = max(np.abs(params[k] - g['param_final/' + k]).max() for k in names)
        # Adam moves each weight by ~lr per step: bf16-rounded gradients of the same sign
        # leave the 3-step trajectory within a fraction of 3 lr
        assert worst < 2e-3, worst
    for k in names:
        np.testing.assert_array_equal(got[0][1][k], got[1][1][k], err_msg=k)


def _gen_worker(rank, world, port, name, dtype, sampler, n, q):
    """Rank-sharded generation (model.shard_generate): each rank generates its contiguous
    rows with the noise of the global rows (Philox, or the reference's torch CPU stream
    drawn for the whole batch on every rank); the gathered batch equals the single-process
    run's bit for bit.  n not divisible by the world size: the rows are padded as
    generate.py pads them, and the noise is drawn for the true n (noise_rows)."""
    try:
        sys.path[:0] = [HERE, os.path.join(HERE, 'golden'),
                        os.path.join(os.path.dirname(HERE),
                                     'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd')]
        os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
        import distributed as D
        import model as M
        import recipe
        import samplernn_hip as H
        from test_gpu_parity import build
        D.init(backend='gloo')
        H.lib()
        cfg = recipe.CONFIGS[name]
        m, _ = build(cfg, recipe.make_weights(cfg, 51),
                     torch.bfloat16 if dtype == 'bf16' else torch.float32)
        n_cond = 2
        cond = recipe.synth_cond((n, n_cond, cfg['cond_dim']), 6)
        spk = np.arange(n) % cfg['spk_dim']
        pad = (-n) % world
        pcond = np.concatenate([cond, np.zeros((pad,) + cond.shape[1:], cond.dtype)])
        pspk = np.concatenate([spk, np.zeros(pad, spk.dtype)])
        torch.manual_seed(7)
        out = M.shard_generate(M.Generator(m, True), n + pad, pcond, pspk, 99, sampler=sampler,
                               noise_rows=n)[:n]
        full = None
        if rank == 0:
            torch.manual_seed(7)
            full = M.Generator(m, True)(n, 0, cond, spk, sampler=sampler, seed=99)
            full = full.numpy()
        q.put((rank, out.numpy(), full, None))
        D.barrier()
        import torch.distributed as dist
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, None, None, traceback.format_exc()))
        raise


@pytest.mark.parametrize('name,dtype,sampler,n', [('t3', 'fp32', 'philox', 16),
                                                  ('big', 'bf16', 'philox', 16),
                                                  ('t3', 'fp32', 'torch', 16),
                                                  ('big', 'fp32', 'torch', 16),
                                                  ('t3', 'fp32', 'torch', 15),
                                                  ('t3', 'fp32', 'philox', 15)])
def test_sharded_generation_reproduces_single_process(hip, name, dtype, sampler, n):
    got = _spawn(_gen_worker, (name, dtype, sampler, n))
    full = got[0][1]
    for rank in (0, 1):
        assert np.array_equal(got[rank][0], full), rank


def _graph_dp_worker(port, zero, q):
    """ONE rank over nccl (RCCL) with the bucket path forced (SRNN_DP_FORCE=1) and graph mode
    under DP (SRNN_GRAPH_DP=1): the Trainer captures the whole data-parallel step -- the
    bucket all-reduces, or with zero the reduce-scatters, the sharded clamp + Adam and the
    parameter all-gathers of ZeRO-1 -- into the HIP graph and replays it.  Returns the losses, the final parameters and the
    number of replayed steps; the caller compares them with a plain single-process run."""
    try:
        sys.path[:0] = [HERE, os.path.join(HERE, 'golden'),
                        os.path.join(os.path.dirname(HERE),
                                     'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd')]
        os.environ.update(SRNN_DP_FORCE='1', SRNN_GRAPH_DP='1', SRNN_DP_ZERO='1' if zero else '0')
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group('nccl', init_method='tcp://127.0.0.1:%d' % port, rank=0,
                                world_size=1, device_id=torch.device('cuda', 0))
        out = _run_graph_steps(dp=True)
        q.put(out + (None,))
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((None, None, None, traceback.format_exc()))
        raise


def _run_graph_steps(dp):
    import distributed as D
    import nn as snn
    import optim
    import recipe
    import samplernn_hip as H
    from conftest import golden
    from test_gpu_parity import build
    from trainer import Trainer
    H.lib()
    g = golden('tbptt_t3')
    cfg = recipe.CONFIGS['t3']
    m, pred = build(cfg, recipe.make_weights(cfg, int(g['weight_seed'])), torch.bfloat16)
    sync = D.GradAllReduce(bucket_mb=0.01, overlap_groups=D.readiness_groups(pred)) if dp \
        else None
    opt = optim.gradient_clipping(torch.optim.Adam(pred.parameters(), lr=1e-3), grad_sync=sync)
    B = int(g['B'])
    losses = []
    criterion = snn.sequence_nll_loss_bits      # (graph mode captures only the bits loss)
    dev = 'cuda'
    chunks = [(torch.from_numpy(g['input_%d' % s]).to(dev),
               torch.tensor([int(g['reset_%d' % s])] * B),
               torch.from_numpy(g['target_%d' % s]).to(dev),
               torch.from_numpy(g['cond_%d' % s]).to(dev),
               torch.from_numpy(g['spk_%d' % s]).to(dev)) for s in range(3)]
    # reset chunk, then 5 carried chunks: the carried kind is captured on its 2nd occurrence
    data = [chunks[0]] + [(c[0], torch.zeros(B, dtype=torch.long)) + c[2:]
                          for c in (chunks[1], chunks[2]) * 3][:5]

    class _Loss:
        trigger_interval = [(1, 'iteration')]

        def register(self, tr):
            pass

        def iteration(self, it, inp, tgt, out, loss):
            losses.append(float(loss))
    tr = Trainer(pred, criterion, opt, data, True, None)
    tr.register_plugin(_Loss())
    tr.run(1)
    torch.cuda.synchronize()
    H.check_persistent_errors()
    # (numpy, not tensors: CPU tensors sent through a multiprocessing queue are shared by
    #  file descriptor, which dies with the worker)
    params = {k: p.detach().cpu().numpy().copy() for k, p in pred.named_parameters()}
    return losses, params, tr.graph_steps


@pytest.mark.parametrize('zero', [False, True])
def test_graph_captured_dp_step_over_rccl(hip, zero):
    """The data-parallel step (bucket all-reduces, or ZeRO-1's reduce-scatter / sharded Adam /
    all-gather, over RCCL) captured in the HIP graph and replayed equals the single-process
    bf16 step bit for bit (one rank: the SUM of one shard is the gradient itself, scale 1)."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    p = ctx.Process(target=_graph_dp_worker, args=(_free_port(), zero, q))
    p.start()
    losses, params, replays, err = q.get(timeout=150)
    p.join(timeout=30)
    assert err is None, err
    assert p.exitcode == 0
    assert replays >= 3, replays
    ref_losses, ref_params, ref_replays = _run_graph_steps(dp=False)
    assert ref_replays >= 3
    assert losses == ref_losses
    for k in ref_params:
        np.testing.assert_array_equal(params[k], ref_params[k], err_msg=k)
