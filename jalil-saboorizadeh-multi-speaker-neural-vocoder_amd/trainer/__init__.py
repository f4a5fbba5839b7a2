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
"""
import heapq
import time

import torch

import samplernn_hip as H


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

    def register_plugin(self, plugin):
        plugin.register(self)
        intervals = plugin.trigger_interval
        if not isinstance(intervals, list):
            intervals = [intervals]
        for (duration, unit) in intervals:
            queue = self.plugin_queues[unit]
            queue.append((duration, len(queue), plugin))

    def call_plugins(self, queue_name, time, *args):
        args = (time,) + args
        queue = self.plugin_queues[queue_name]
        if len(queue) == 0:
            return
        while queue[0][0] <= time:
            plugin = queue[0][2]
            getattr(plugin, queue_name)(*args)
            for trigger in plugin.trigger_interval:
                if trigger[1] == queue_name:
                    interval = trigger[0]
            new_item = (time + interval, queue[0][1], plugin)
            heapq.heappushpop(queue, new_item)

    def run(self, epochs=1):
        for q in self.plugin_queues.values():
            heapq.heapify(q)
        for self.epochs in range(self.epochs + 1, self.epochs + int(epochs) + 1):
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
