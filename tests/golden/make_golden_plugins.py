"""Recording plugins for the plugin-schedule fixture (tests/golden/plugin_order.npz):
used by make_golden.py with the reference's Trainer and by tests/test_cpu_host.py with ours."""


class RecPlugin:
    """A plugin that records (unit, time, id) whenever the Trainer fires it."""

    def __init__(self, pid, triggers, log):
        self.pid, self.trigger_interval, self.log = pid, triggers, log

    def register(self, trainer):
        pass

    def _fire(self, unit, time):
        self.log.append((unit, time, self.pid))

    def iteration(self, time, *a):
        self._fire(0, time)

    def epoch(self, time, *a):
        self._fire(1, time)

    def batch(self, time, *a):
        self._fire(2, time)

    def update(self, time, *a):
        self._fire(3, time)


PLUGIN_TRIGGERS = [[(1, 'iteration')], [(3, 'iteration'), (1, 'epoch')],
                   [(2, 'iteration'), (2, 'epoch')], [(3, 'iteration'), (5, 'iteration')],
                   [(2, 'batch'), (1, 'update')], [(1, 'iteration'), (4, 'update')],
                   [(2, 'iteration')]]
