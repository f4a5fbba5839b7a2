"""Drop-in for the reference's trainer/__init__.py (trainer/__init__.py:1-117).

Same Trainer API (constructor, register_plugin, call_plugins, run, train, plugin
queues 'iteration' / 'epoch' / 'batch' / 'update', stats, iterations, epochs).  The
TBPTT step itself is unchanged in structure -- reset flag, device copies, closure
(forward, criterion, backward), optimizer.step(closure) -- and runs on the HIP model.
zero_grad keeps torch-0.4 semantics (grads zero-filled, never None) so the reference's
gradient_clipping never meets a None grad.

The per-iteration check of the persistent sweeps' failure flag is lagged by one step and
needs no device synchronisation (samplernn_hip.PersistentErrorWatch): the host keeps
enqueuing while the GPU runs; a failure raises one iteration later (or at the epoch's end),
after the Adam step counters of the skipped updates are rolled back.

Graph mode (SRNN_GRAPH=1, the default on a GPU): the whole TBPTT step -- forward, loss,
backward, clip + Adam -- is captured once per step kind into a HIP graph and replayed, so
the host enqueues one graph launch instead of every kernel.  A step kind is (fresh hidden
state or carried, batch shapes, what the optimizer baked in: learning rates and the
addresses of parameters / moments / bf16 copies); the first occurrence of a kind runs
eagerly (it is also the warm-up that sizes every workspace), the second is captured and
replayed, later ones replay.  The batch is copied into static input buffers and the carried
hidden state lives in static buffers the graph reads and rewrites; the Adam step count is
read from a device counter (optim.DeviceSteps) so replays keep the bias correction exact.
Anything a captured step cannot honour falls back to the eager step: roofline probes on
(bench.py's per-kernel timing), a data-parallel gradient hook over gloo (RCCL collectives
are captured; SRNN_GRAPH_DP=0 keeps any DP step eager), a model without the Predictor's
hidden-state carry, and any criterion other than the
reference's `nn.sequence_nll_loss_bits` (user code runs inside the capture and may
synchronise, e.g. read the loss with .item(); SRNN_GRAPH=force captures it anyway, and a
capture that fails rolls the step's host state back and runs it eagerly).  After a replay
every parameter's .grad is the graph's gradient tensor, holding this step's clamped gradient
as after an eager step (optim.py:11-13).
"""
import heapq
import os
import time

import torch

import samplernn_hip as H

GRAPHS = os.environ.get('SRNN_GRAPH', '1') != '0'
FORCE = os.environ.get('SRNN_GRAPH', '1') == 'force'


def _capture_agreed(opt, ok):
    """True iff the capture succeeded on every rank of the optimizer's data-parallel group
    (MIN all-reduce of the local outcome, outside any capture); `ok` alone without one."""
    sync = getattr(opt, 'grad_sync', None)
    if sync is None:
        return ok
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return ok
    grp = getattr(sync, 'group', None)
    if dist.get_world_size(grp) <= 1:
        return ok
    dev = 'cuda' if dist.get_backend(grp) == 'nccl' else 'cpu'
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=grp)
    return bool(flag.item())


class _StepGraph:
    """One captured TBPTT step: the graph, its static inputs and outputs."""

    def __init__(self, x, tgt, cond, spk):
        self.x, self.tgt, self.cond, self.spk = x, tgt, cond, spk
        self.graph = None
        self.out = self.loss = None
        self.grads = []             # (parameter, the graph's gradient tensor or None)
        self.replays = 0


class Trainer(object):

    def __init__(self, model, criterion, optimizer, dataset, cuda, writer, scheduler=None):
        self.model = model
        self.criterion = criterion
        self.optimizer = optimizer
        self.scheduler = scheduler
        self.dataset = dataset
        self.cuda = cuda
        self.iterations = 0
        self.epochs = 0
        self.stats = {}
        self.plugin_queues = {
            'iteration': [],
            'epoch': [],
            'batch': [],
            'update': [],
        }
        self.writer = writer
        self._watch = None
        self.enqueue_s = 0.0        # host seconds spent enqueuing steps (bench.py)
        self.graphs = {}            # step kind -> _StepGraph (graph mode)
        self._seen = set()          # step kinds that ran eagerly once
        self._hbuf = {}             # (tier index, rows) -> static carried hidden state
        self.graph_steps = 0        # steps replayed from a graph (tests, bench.py)
        self._no_graph = set()      # step kinds whose capture failed

    # ---- plugin schedule (trainer/__init__.py:28-60).  One min-heap per unit ('iteration',
    # 'epoch', 'batch', 'update') of (next due time, registration order within the unit,
    # plugin): a plugin first fires when the unit's clock reaches its interval, and after
    # firing at time t it is due again at t + interval (of its LAST trigger for that unit);
    # plugins due at the same time fire in registration order.  The lists stay reachable as
    # self.plugin_queues, as in the reference.
    @staticmethod
    def _triggers(plugin):
        ti = plugin.trigger_interval
        return ti if isinstance(ti, list) else [ti]

    def register_plugin(self, plugin):
        plugin.register(self)
        for every, unit in self._triggers(plugin):
            heap = self.plugin_queues[unit]
            heapq.heappush(heap, (every, len(heap), plugin))

    def call_plugins(self, queue_name, time, *args):
        heap = self.plugin_queues[queue_name]
        while heap and heap[0][0] <= time:
            _, order, plugin = heap[0]
            getattr(plugin, queue_name)(time, *args)
            every = [n for n, unit in self._triggers(plugin) if unit == queue_name][-1]
            heapq.heapreplace(heap, (time + every, order, plugin))

    def run(self, epochs=1):
        for heap in self.plugin_queues.values():
            heapq.heapify(heap)        # (a no-op: registration keeps each list a heap)
        first = self.epochs + 1
        for self.epochs in range(first, first + int(epochs)):
            self.train()
            if self.scheduler is not None:
                self.scheduler.step()
            self.call_plugins('epoch', self.epochs)

    def _zero_grad(self):
        if hasattr(self.optimizer, 'grad_sync'):    # optim.gradient_clipping wrapper
            self.optimizer.zero_grad()
            return
        try:
            self.optimizer.zero_grad(set_to_none=False)
        except TypeError:
            self.optimizer.zero_grad()

    def _rollback(self, k):
        fn = getattr(self.optimizer, 'rollback_steps', None)
        if fn is not None:
            fn(k)

    def train(self):
        if self.cuda and self._watch is None:
            self._watch = H.PersistentErrorWatch()
        for (self.iterations, data) in enumerate(self.dataset, self.iterations + 1):
            t_enq = time.perf_counter()
            inputs = data[0]
            reset = data[1]
            batch_target = data[2]
            reset = bool(reset[0] == 1) if torch.is_tensor(reset) or isinstance(reset, (list, tuple)) \
                else bool(reset)
            batch_inputs = (inputs, reset)
            batch_cond = data[3]
            batch_spk = data[4]

            self.call_plugins('batch', self.iterations, batch_inputs, batch_target, batch_cond,
                              batch_spk)

            def wrap(input):
                if torch.is_tensor(input) and self.cuda:
                    input = input.cuda(non_blocking=True)
                return input
            batch_inputs = list(map(wrap, batch_inputs))
            if self.cuda:
                batch_target = batch_target.cuda(non_blocking=True)
                batch_cond = batch_cond.cuda(non_blocking=True)
                batch_spk = batch_spk.cuda(non_blocking=True)

            kind = self._step_kind(batch_inputs, batch_target, batch_cond, batch_spk)
            plugin_data = None
            if kind is not None and (kind in self.graphs or kind in self._seen):
                plugin_data = self._graph_step(kind, batch_inputs, batch_target, batch_cond,
                                               batch_spk)
            if plugin_data is not None:
                self.enqueue_s += time.perf_counter() - t_enq
                self._watch.step(self._rollback)
                self.call_plugins('iteration', self.iterations, batch_inputs, batch_target,
                                  *plugin_data)
                self.call_plugins('update', self.iterations, self.model)
                continue
            if kind is not None:
                self._seen.add(kind)
            plugin_data = [None, None]

            def closure():
                batch_output = self.model(*batch_inputs, batch_cond, batch_spk, self.writer,
                                          self.iterations)
                loss = self.criterion(batch_output, batch_target)
                loss.backward()
                if plugin_data[0] is None:
                    plugin_data[0] = batch_output.data
                    plugin_data[1] = loss.data
                return loss

            self._zero_grad()
            self.optimizer.step(closure)
            self.enqueue_s += time.perf_counter() - t_enq
            if self.cuda:
                self._watch.step(self._rollback)
            self.call_plugins('iteration', self.iterations, batch_inputs, batch_target,
                              *plugin_data)
            self.call_plugins('update', self.iterations, self.model)
        if self.cuda:
            self._watch.flush(self._rollback)

    # ------------------------------------------------------------------ graph mode
    def _step_kind(self, batch_inputs, target, cond, spk):
        """The key of a capturable step, or None when this step must run eagerly."""
        if not (GRAPHS and self.cuda) or H.ROOF_EVENTS is not None:
            return None
        import nn as snn
        if self.criterion is not snn.sequence_nll_loss_bits and not FORCE:
            return None
        opt = self.optimizer
        if not (hasattr(opt, 'graph_ready') and opt.graph_ready()):
            return None
        hs = getattr(self.model, 'hidden_states', None)
        rnns = getattr(getattr(self.model, 'model', None), 'frame_level_rnns', None)
        if hs is None or rnns is None:
            return None
        inputs, reset = batch_inputs
        fresh = bool(reset) or all(h is None for h in hs.values())
        if not fresh and any(hs.get(r) is None for r in rnns):
            return None
        ts = (inputs, target, cond, spk)
        if not all(torch.is_tensor(t) and t.is_cuda for t in ts):
            return None
        kind = (fresh,) + tuple((tuple(t.shape), t.dtype) for t in ts) + \
            (opt.graph_signature(),)
        return None if kind in self._no_graph else kind

    def _hidden_bufs(self, rows):
        """Static carried hidden state per tier (n_rnn, rows, dim) fp32."""
        bufs = []
        dev = self.optimizer.dsteps.t.device
        for i, rnn in enumerate(self.model.model.frame_level_rnns):
            b = self._hbuf.get((i, rows))
            if b is None:
                b = torch.zeros(rnn.n_rnn, rows, rnn.dim, device=dev)
                self._hbuf[(i, rows)] = b
            bufs.append(b)
        return bufs

    def _graph_step(self, kind, batch_inputs, target, cond, spk):
        """Replay the captured step of this kind (capturing it first if needed); returns the
        static (output, loss) handed to the plugins."""
        model = self.model
        rnns = model.model.frame_level_rnns
        fresh = kind[0]
        inputs = batch_inputs[0]
        bufs = self._hidden_bufs(inputs.shape[0])
        sg = self.graphs.get(kind)
        if not fresh:
            for rnn, b in zip(rnns, bufs):       # the carried state into the static buffers
                h = model.hidden_states[rnn]
                if h is not b:
                    if h.shape != b.shape or h.dtype != b.dtype:
                        raise RuntimeError('graph mode: carried hidden state %s %s, buffer %s'
                                           % (tuple(h.shape), h.dtype, tuple(b.shape)))
                    b.copy_(h)
                    model.hidden_states[rnn] = b
        if sg is None:
            sg = self._capture(kind, inputs, target, cond, spk, bufs)
            if sg is None:
                return None                       # capture failed: run the step eagerly
        else:
            sg.x.copy_(inputs)
            sg.tgt.copy_(target)
            sg.cond.copy_(cond)
            sg.spk.copy_(spk)
            self.optimizer.before_replay()
            sg.graph.replay()
            self.optimizer.after_replay()
            for p, gr in sg.grads:
                p.grad = gr
        sg.replays += 1
        self.graph_steps += 1
        for rnn, b in zip(rnns, bufs):
            model.hidden_states[rnn] = b
        return [sg.out, sg.loss]

    def _capture(self, kind, inputs, target, cond, spk, bufs):
        """Capture one step (its Python side effects -- Adam step counts, hidden-state
        bookkeeping -- happen once, for the replay that follows)."""
        # graphs baked against an older optimizer state are dead: free their memory
        self.graphs = {k: g for k, g in self.graphs.items() if k[-1] == kind[-1]}
        sg = _StepGraph(inputs.clone(), target.clone(), cond.clone(), spk.clone())
        model, fresh = self.model, kind[0]
        rnns = model.model.frame_level_rnns
        self._zero_grad()
        self.optimizer.before_replay()
        # host state the capture's Python side effects change, for a roll-back on failure
        saved_hidden = dict(model.hidden_states)
        opt = self.optimizer
        saved_steps = [(st, st['step'].clone()) for st in opt.state.values() if 'step' in st]
        saved_mirror = list(opt.dsteps.mirror)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        out_loss = [None, None]

        def closure():
            out = model(sg.x, fresh, sg.cond, sg.spk, self.writer, self.iterations)
            loss = self.criterion(out, sg.tgt)
            loss.backward()
            out_loss[0], out_loss[1] = out.data, loss.data
            return loss
        err = None
        try:
            # a private memory pool per step kind; thread-local capture mode, so other
            # threads' HIP calls (the RCCL process group's watchdog querying its events under
            # data parallelism) do not invalidate the capture
            with torch.cuda.graph(g, capture_error_mode='thread_local'):
                self.optimizer.step(closure)
                for rnn, b in zip(rnns, bufs):
                    h = model.hidden_states[rnn]
                    if h.shape != b.shape or h.dtype != b.dtype:
                        raise RuntimeError('graph mode: new hidden state %s %s, buffer %s'
                                           % (tuple(h.shape), h.dtype, tuple(b.shape)))
                    b.copy_(h)
        except Exception as e:  # noqa: BLE001 -- any capture failure: roll back, run eagerly
            err = e
        # under data parallelism every rank must take the same path after a capture attempt
        # (one rank replaying captured collectives while another issues them eagerly would
        # desynchronise the communicator): the ranks agree on the outcome, and a failure on
        # any rank rolls every rank back to the eager step
        if not _capture_agreed(opt, err is None) and err is None:
            err = RuntimeError('capture failed on another rank')
        if err is not None:
            import warnings
            e = err
            torch.cuda.synchronize()
            model.hidden_states.clear()
            model.hidden_states.update(saved_hidden)
            for st, v in saved_steps:
                st['step'] = v
            opt.dsteps.mirror = [None] * len(saved_mirror)   # re-seeded at the next step
            self._zero_grad()
            self._no_graph.add(kind)
            warnings.warn('graph mode: capture failed (%s: %s); this step kind runs eagerly'
                          % (type(e).__name__, e))
            return None
        sg.graph = g
        sg.out, sg.loss = out_loss
        sg.grads = [(p, p.grad) for grp in opt.param_groups for p in grp['params']]
        self.graphs[kind] = sg
        g.replay()
        return sg
