"""Import shims so the reference's own scripts run on this package unchanged.

The reference's train.py / generate.py / trainer/plugins.py import modules this image does
not have (torch 0.4's torch.utils.trainer, tensorboardX, natsort, librosa 0.6).  `install()`
registers stand-ins in sys.modules that map onto this package:

  torch.utils.trainer[.plugins[.plugin|.monitor]] -> trainer.plugins (Plugin, Monitor,
                                                     LossMonitor, Logger)
  tensorboardX.SummaryWriter                      -> torch.utils.tensorboard if importable,
                                                     else a writer that drops everything
  natsort.natsorted                               -> natural sort on digit runs
  librosa.core.load / librosa.load                -> dataset.load_wav (+ resample refused)
  librosa.output.write_wav                        -> dataset.write_wav

Our own train.py / generate.py do not need this; it exists for users who keep running the
reference's scripts with this package first on sys.path:
    python -c "import compat; compat.install(); import runpy; runpy.run_path('train.py', ...)"
"""
import re
import sys
import types


def _natsorted(seq, key=None):
    def k(x):
        s = key(x) if key else x
        return [int(t) if t.isdigit() else t for t in re.split(r'(\d+)', str(s))]
    return sorted(seq, key=k)


class _NullWriter:
    def __init__(self, *a, **kw):
        pass

    def __getattr__(self, name):
        return lambda *a, **kw: None


def install():
    import dataset
    from trainer import plugins as P

    tr = types.ModuleType('torch.utils.trainer')
    trp = types.ModuleType('torch.utils.trainer.plugins')
    trpp = types.ModuleType('torch.utils.trainer.plugins.plugin')
    trpm = types.ModuleType('torch.utils.trainer.plugins.monitor')
    for m in (trp,):
        m.Plugin, m.Monitor, m.LossMonitor, m.Logger = P.Plugin, P.Monitor, P.LossMonitor, P.Logger
    trpp.Plugin = P.Plugin
    trpm.Monitor = P.Monitor
    trp.plugin, trp.monitor = trpp, trpm
    tr.plugins = trp
    sys.modules.setdefault('torch.utils.trainer', tr)
    sys.modules.setdefault('torch.utils.trainer.plugins', trp)
    sys.modules.setdefault('torch.utils.trainer.plugins.plugin', trpp)
    sys.modules.setdefault('torch.utils.trainer.plugins.monitor', trpm)

    tbx = types.ModuleType('tensorboardX')
    try:
        from torch.utils.tensorboard import SummaryWriter
        tbx.SummaryWriter = SummaryWriter
    except Exception:  # tensorboard not installed
        tbx.SummaryWriter = _NullWriter
    sys.modules.setdefault('tensorboardX', tbx)

    ns = types.ModuleType('natsort')
    ns.natsorted = _natsorted
    sys.modules.setdefault('natsort', ns)

    def load(path, sr=None, mono=True, **kw):
        y, rate = dataset.load_wav(path)
        if sr is not None and sr != rate:
            raise NotImplementedError('compat librosa.load: resampling (%d -> %d)' % (rate, sr))
        return y, rate

    lr = types.ModuleType('librosa')
    lrc = types.ModuleType('librosa.core')
    lro = types.ModuleType('librosa.output')
    lrc.load = lr.load = load
    lro.write_wav = dataset.write_wav
    lr.core, lr.output = lrc, lro
    sys.modules.setdefault('librosa', lr)
    sys.modules.setdefault('librosa.core', lrc)
    sys.modules.setdefault('librosa.output', lro)
