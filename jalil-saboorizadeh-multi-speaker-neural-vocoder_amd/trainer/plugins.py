"""Drop-in for the reference's trainer/plugins.py (plugins.py:1-303) plus the
torch.utils.trainer plugin base classes it builds on (removed from PyTorch after 0.4),
restated here so train.py needs no torch 0.4.

Base classes (old torch.utils.trainer.plugins API): Plugin(interval), Monitor (running and
epoch averages, log field templates), LossMonitor, Logger (the tab-separated
'name: value (running)' lines plotlog.py parses, plotlog.py:23-26).

Reference plugins: TrainingLossMonitor, ValidationPlugin (teacher-forced evaluation on the
HIP Predictor, loss read with .item() -- the reference's `loss.data[0]`, plugins.py:88,
fails on torch >= 0.5), AbsoluteTimeMonitor, SaverPlugin (ep{E}-it{I} / best-ep{E}-it{I}
state_dict checkpoints), GeneratorPlugin (device generation + WAV), StatsPlugin (stats.pkl +
svg plots), CometPlugin.

The reference plugins are samplernn-pytorch's (MIT, (c) 2017 Piotr Kozakowski); their names,
checkpoint naming, log-line format and pickle layout are the drop-in contract, restated here
(THIRD_PARTY_NOTICES.md).
"""
import os
import pickle
import time
from collections import defaultdict
from glob import glob

import torch


# ---------------------------------------------------------------- torch.utils.trainer base
class Plugin(object):
    """torch.utils.trainer.plugins.plugin.Plugin: a list of (period, unit) triggers."""

    def __init__(self, interval=None):
        self.trigger_interval = interval if interval is not None else []

    def register(self, trainer):
        raise NotImplementedError


class Monitor(Plugin):
    """torch.utils.trainer.plugins.monitor.Monitor: per-iteration value with an exponential
    running average and an epoch mean; stats[stat_name] holds last / running_avg /
    epoch_mean and the log field templates."""

    stat_name = None

    def __init__(self, running_average=True, epoch_average=True, smoothing=0.7,
                 precision=None, number_format=None, unit=''):
        precision = 4 if precision is None else precision
        number_format = ':' + ('.{}f'.format(precision) if number_format is None
                               else number_format)
        super().__init__([(1, 'iteration'), (1, 'epoch')])
        self.smoothing = smoothing
        self.with_running_average = running_average
        self.with_epoch_average = epoch_average
        self.log_format = number_format
        self.log_unit = unit
        self.log_epoch_fields = None
        self.log_iter_fields = ['{last' + number_format + '}' + unit]
        if running_average:
            self.log_iter_fields.append(' ({running_avg' + number_format + '}' + unit + ')')
        if epoch_average:
            self.log_epoch_fields = ['{epoch_mean' + number_format + '}' + unit]

    def register(self, trainer):
        self.trainer = trainer
        stats = trainer.stats.setdefault(self.stat_name, {})
        stats['log_format'] = self.log_format
        stats['log_unit'] = self.log_unit
        stats['log_iter_fields'] = self.log_iter_fields
        if self.with_epoch_average:
            stats['log_epoch_fields'] = self.log_epoch_fields
            stats['epoch_stats'] = (0, 0)

    def _get_value(self, *args):
        raise NotImplementedError

    def iteration(self, *args):
        stats = self.trainer.stats.setdefault(self.stat_name, {})
        stats['last'] = self._get_value(*args)
        if self.with_epoch_average:
            s, n = stats['epoch_stats']
            stats['epoch_stats'] = (s + stats['last'], n + 1)
        if self.with_running_average:
            prev = stats.get('running_avg', 0)
            stats['running_avg'] = prev * self.smoothing + stats['last'] * (1 - self.smoothing)

    def epoch(self, idx):
        stats = self.trainer.stats.setdefault(self.stat_name, {})
        if self.with_epoch_average:
            s, n = stats['epoch_stats']
            stats['epoch_mean'] = s / n if n else float('nan')
            stats['epoch_stats'] = (0, 0)


class LossMonitor(Monitor):
    """torch.utils.trainer.plugins.LossMonitor: the iteration's loss (a scalar tensor)."""

    stat_name = 'loss'

    def _get_value(self, iteration, input, target, output, loss):
        return float(loss.item() if torch.is_tensor(loss) else loss)


class Logger(Plugin):
    """torch.utils.trainer.plugins.Logger: one tab-separated line per iteration
    ('training_loss: 7.1234 (7.3456)\\ttime: 12s'), an epoch summary between separators;
    columns keep the widest value seen so far."""

    separator = '#' * 80

    def __init__(self, fields, interval=None):
        super().__init__(interval if interval is not None else [(1, 'iteration'), (1, 'epoch')])
        self.field_widths = defaultdict(lambda: defaultdict(int))
        self.fields = [f.split('.') for f in fields]

    def register(self, trainer):
        self.trainer = trainer

    def log(self, msg):
        print(msg)

    def _outputs(self, field, key, parent, stat, require_dict):
        if isinstance(stat, dict):
            name = stat.get('log_name', '.'.join(field))
            return name, [f.format(**stat) for f in stat.get(key, [])]
        if require_dict:
            return '', []
        fmt = '{' + parent.get('log_format', '') + '}' + parent.get('log_unit', '')
        return '.'.join(field), [fmt.format(stat)]

    def _log_all(self, key, prefix=None, suffix=None, require_dict=False):
        results = []
        for idx, field in enumerate(self.fields):
            parent, stat = None, self.trainer.stats
            try:
                for f in field:
                    parent, stat = stat, stat[f]
            except KeyError:
                continue
            name, out = self._outputs(field, key, parent, stat, require_dict)
            if not out:
                continue
            widths = self.field_widths[idx]
            for j, o in enumerate(out):
                if len(o) < widths[j]:
                    out[j] = o + ' ' * (widths[j] - len(o))
                else:
                    widths[j] = len(o)
            results.append((name, out))
        if not results:
            return
        line = '\t'.join('{}: {}'.format(n, ' '.join(o)) for n, o in results)
        if prefix is not None:
            self.log(prefix)
        self.log(line)
        if suffix is not None:
            self.log(suffix)

    def iteration(self, *args):
        self._log_all('log_iter_fields')

    def epoch(self, epoch_idx):
        self._log_all('log_epoch_fields', prefix=self.separator + '\nEpoch summary:',
                      suffix=self.separator, require_dict=True)


# ---------------------------------------------------------------- reference plugins
class TrainingLossMonitor(LossMonitor):
    """plugins.py:22-24.  Under row-sharded data parallelism (distributed.py) the logged value
    is the mean of the ranks' shard losses = the full-batch loss the single-process run logs."""

    stat_name = 'training_loss'

    def _get_value(self, iteration, input, target, output, loss):
        import distributed
        return distributed.mean_over_ranks(super()._get_value(iteration, input, target, output,
                                                              loss))


class ValidationPlugin(Plugin):
    """plugins.py:27-96: teacher-forced loss over the validation and test loaders each
    epoch (model in eval mode, no autograd graph); row shards summed over ranks under DP."""

    def __init__(self, val_dataset, test_dataset, writer):
        super().__init__([(1, 'epoch')])
        self.val_dataset = val_dataset
        self.test_dataset = test_dataset
        self.writer = writer

    def register(self, trainer):
        self.trainer = trainer
        trainer.stats.setdefault('validation_loss', {})['log_epoch_fields'] = ['{last:.4f}']
        trainer.stats.setdefault('test_loss', {})['log_epoch_fields'] = ['{last:.4f}']

    def epoch(self, idx):
        self.trainer.model.eval()
        self.trainer.stats.setdefault('validation_loss', {})['last'] = \
            self._evaluate(self.val_dataset, idx)
        self.trainer.stats.setdefault('test_loss', {})['last'] = \
            self._evaluate(self.test_dataset, idx)
        self.trainer.model.train()

    def _evaluate(self, dataset, idx):
        loss_sum, n_examples = 0.0, 0
        with torch.no_grad():
            for data in dataset:
                inputs, reset, target, cond, spk = data[:5]
                reset = bool(reset[0] == 1) if torch.is_tensor(reset) or \
                    isinstance(reset, (list, tuple)) else bool(reset)
                if self.trainer.cuda:
                    inputs, target = inputs.cuda(), target.cuda()
                    cond, spk = cond.cuda(), spk.cuda()
                out = self.trainer.model(inputs, reset, cond, spk, self.writer, idx)
                loss = self.trainer.criterion(out, target)
                bs = target.size(0)
                loss_sum += loss.item() * bs
                n_examples += bs
        # under data parallelism each rank saw its row shard: sum (loss, rows) over ranks so
        # every rank -- and SaverPlugin's best-checkpoint choice -- sees the full-batch value
        import distributed
        # a persistent sweep that gave up a hand-off during evaluation makes the loss invalid:
        # its flag is summed with the loss over ranks, so every rank raises before the value
        # is logged or SaverPlugin picks a checkpoint by it
        flag = _persistent_flag() if self.trainer.cuda else 0.0
        loss_sum, n_examples, flag = distributed.sum_over_ranks([loss_sum, n_examples, flag])
        if flag > 0:
            import samplernn_hip as H
            try:
                H.check_persistent_errors()          # clears this rank's flag
            except RuntimeError:
                pass
            raise RuntimeError('persistent GRU sweep gave up a hand-off during evaluation -- '
                               'the evaluation loss is invalid')
        return loss_sum / n_examples if n_examples else float('nan')


def _persistent_flag():
    """This rank's persistent-sweep failure flag as 0.0 / 1.0 (synchronises)."""
    import samplernn_hip as H
    t = torch.zeros(1, device='cuda')
    H.lib().call('srnn_persistent_flag_to_f32', H.ptr(t), H.stream())
    return float(t.item())


class AbsoluteTimeMonitor(Monitor):
    """plugins.py:99-115: seconds since the first iteration."""

    stat_name = 'time'

    def __init__(self, *args, **kwargs):
        kwargs.setdefault('unit', 's')
        kwargs.setdefault('precision', 0)
        kwargs.setdefault('running_average', False)
        kwargs.setdefault('epoch_average', False)
        super().__init__(*args, **kwargs)
        self.start_time = None

    def _get_value(self, *args):
        if self.start_time is None:
            self.start_time = time.time()
        return time.time() - self.start_time


class SaverPlugin(Plugin):
    """plugins.py:118-164: last and best (by validation loss) state_dict checkpoints."""

    last_pattern = 'ep{}-it{}'
    best_pattern = 'best-ep{}-it{}'

    def __init__(self, checkpoints_path, keep_old_checkpoints):
        super().__init__([(1, 'epoch')])
        self.checkpoints_path = checkpoints_path
        self.keep_old_checkpoints = keep_old_checkpoints
        self._best_val_loss = float('+inf')

    def register(self, trainer):
        self.trainer = trainer

    def epoch(self, epoch_index):
        if not self.keep_old_checkpoints:
            self._clear(self.last_pattern.format('*', '*'))
        torch.save(self.trainer.model.state_dict(),
                   os.path.join(self.checkpoints_path,
                                self.last_pattern.format(epoch_index, self.trainer.iterations)))
        cur = self.trainer.stats['validation_loss']['last']
        if cur < self._best_val_loss:
            self._clear(self.best_pattern.format('*', '*'))
            torch.save(self.trainer.model.state_dict(),
                       os.path.join(self.checkpoints_path,
                                    self.best_pattern.format(epoch_index,
                                                             self.trainer.iterations)))
            self._best_val_loss = cur

    def _clear(self, pattern):
        for name in glob(os.path.join(self.checkpoints_path, pattern)):
            os.remove(name)


class GeneratorPlugin(Plugin):
    """plugins.py:167-190: unconditioned-length samples each epoch (peak-normalised WAV).
    The reference calls Generator without cond/spk (which its own Generator rejects);
    here cond defaults to zeros for sample_length / lookback frames and speaker 0."""

    pattern = 'ep{}-s{}.wav'

    def __init__(self, samples_path, n_samples, sample_length, sample_rate, cond=None, spk=0):
        super().__init__([(1, 'epoch')])
        self.samples_path = samples_path
        self.n_samples = n_samples
        self.sample_length = sample_length
        self.sample_rate = sample_rate
        self.cond = cond
        self.spk = spk

    def register(self, trainer):
        from model import Generator
        self.model = trainer.model.model
        self.generate = Generator(self.model, trainer.cuda)

    def epoch(self, epoch_index):
        from dataset import write_wav
        import numpy as np
        cond = self.cond
        if cond is None:
            n_cond = max(1, self.sample_length // self.model.lookback)
            cond = np.zeros((n_cond, self.model.cond_dim), dtype=np.float32)
        samples = self.generate(self.n_samples, self.sample_length, cond, self.spk)
        samples = samples.cpu().float().numpy()
        for i in range(self.n_samples):
            write_wav(os.path.join(self.samples_path, self.pattern.format(epoch_index, i + 1)),
                      samples[i, :], sr=self.sample_rate, norm=True)


class StatsPlugin(Plugin):
    """plugins.py:193-280: iteration / epoch stat histories pickled to stats.pkl, plots."""

    data_file_name = 'stats.pkl'
    plot_pattern = '{}.svg'

    def __init__(self, results_path, iteration_fields, epoch_fields, plots):
        super().__init__([(1, 'iteration'), (1, 'epoch')])
        self.results_path = results_path
        self.iteration_fields = self._fields_to_pairs(iteration_fields)
        self.epoch_fields = self._fields_to_pairs(epoch_fields)
        self.plots = plots
        self.data = {
            'iterations': {f: [] for f in self.iteration_fields + [('iteration', 'last')]},
            'epochs': {f: [] for f in self.epoch_fields + [('iteration', 'last')]},
        }

    def register(self, trainer):
        self.trainer = trainer

    def iteration(self, *args):
        for (field, stat) in self.iteration_fields:
            self.data['iterations'][field, stat].append(self.trainer.stats[field][stat])
        self.data['iterations']['iteration', 'last'].append(self.trainer.iterations)

    def epoch(self, epoch_index):
        for (field, stat) in self.epoch_fields:
            self.data['epochs'][field, stat].append(self.trainer.stats[field][stat])
        self.data['epochs']['iteration', 'last'].append(self.trainer.iterations)
        with open(os.path.join(self.results_path, self.data_file_name), 'wb') as f:
            pickle.dump(self.data, f)
        try:
            import matplotlib
            matplotlib.use('Agg')
            from matplotlib import pyplot
        except ImportError:
            return
        for name, info in self.plots.items():
            x_field = self._field_to_pair(info['x'])
            y_fields = info.get('ys', [info.get('y')])
            labels = [' '.join(y) if isinstance(y, tuple) else y for y in y_fields]
            y_fields = self._fields_to_pairs(y_fields)
            formats = info.get('formats', [''] * len(y_fields))
            pyplot.gcf().clear()
            for y_field, fmt, label in zip(y_fields, formats, labels):
                part = 'iterations' if y_field in self.iteration_fields else 'epochs'
                pyplot.plot(self.data[part][x_field], self.data[part][y_field], fmt, label=label)
            if info.get('log_y'):
                pyplot.yscale('log')
            pyplot.legend()
            pyplot.savefig(os.path.join(self.results_path, self.plot_pattern.format(name)))

    @staticmethod
    def _field_to_pair(field):
        return field if isinstance(field, tuple) else (field, 'last')

    @classmethod
    def _fields_to_pairs(cls, fields):
        return [cls._field_to_pair(f) for f in fields]


class CometPlugin(Plugin):
    """plugins.py:283-303."""

    def __init__(self, experiment, fields):
        super().__init__([(1, 'epoch')])
        self.experiment = experiment
        self.fields = [f if isinstance(f, tuple) else (f, 'last') for f in fields]

    def register(self, trainer):
        self.trainer = trainer

    def epoch(self, epoch_index):
        for (field, stat) in self.fields:
            self.experiment.log_metric(field, self.trainer.stats[field][stat])
        self.experiment.log_epoch_end(epoch_index)
