"""Drop-in for the reference's train.py (train.py:1-458): the TBPTT training CLI.

Same arguments, defaults, experiment tag / results layout (results/<tag>/{checkpoints,
samples,log}), checkpoint names and resume rule, optimizer (Adam + optional
MultiStepLR([15, 35], 0.1) + gradient_clipping) and plugins, built on this package's HIP
model and the FolderDataset stream layout.  Differences, by design:

  * no tensorboardX / natsort / torch.utils.trainer imports (writer = None unless
    tensorboard is importable; checkpoints sorted naturally by (epoch, iteration));
  * multi-GPU data parallelism when launched by torchrun (one process per GPU, RCCL):
    every rank reads the same full-batch DataLoader and keeps its contiguous stream rows
    (distributed.shard_rows); gradients are averaged before the clamp;
    only rank 0 logs and checkpoints.
  * --compute_dtype bf16 runs the MFMA GEMMs in bf16 (fp32 master weights), the bench's
    TBPTT mode; the default fp32 is the reference-parity mode.

  python train.py --exp NAME --frame_sizes 16 4 --dataset wav/ [--cond_set cond/] ...
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 train.py ...   (row-sharded DP)
"""
import argparse
import os
import random
import re
import shutil
import sys
from glob import glob

import numpy as np
import torch

import distributed as dist_mod
from dataset import FolderDataset
from model import SampleRNN, Predictor
from nn import sequence_nll_loss_bits
from optim import gradient_clipping
from trainer import Trainer
from trainer.plugins import (AbsoluteTimeMonitor, Logger, SaverPlugin, StatsPlugin,
                             TrainingLossMonitor, ValidationPlugin)

default_params = {
    # model parameters
    'n_rnn': 1,
    'dim': 1024,
    'learn_h0': True,
    'ulaw': True,
    'q_levels': 256,
    'weight_norm': False,
    'seq_len': 1040,
    'batch_size': 128,
    'look_ahead': False,
    'qrnn': False,
    'cond_dim': 43,         # 40 MFCC + LF0 + FV + U/V (Ahocoder)
    'cond_len': 80,         # one conditioning frame per 80 samples (5 ms at 16 kHz)
    'norm_ind': True,
    'static_spk': False,
    # training parameters
    'keep_old_checkpoints': False,
    'datasets_path': 'datasets',
    'cond_path': 'datasets',
    'results_path': 'results',
    'dataset': 'wav/',
    'cond_set': 'cond/',
    'epoch_limit': 1000,
    'learning_rate': 1e-3,
    'resume': True,
    'sample_rate': 16000,
    'n_samples': 1,
    'sample_length': 80000,
    'loss_smoothing': 0.99,
    'seed': 77977,
    'model': None,
    'scheduler': False,
    'compute_dtype': 'fp32',
}
tag_params = [
    'exp', 'frame_sizes', 'n_rnn', 'dim', 'learn_h0', 'ulaw', 'q_levels', 'seq_len', 'look_ahead',
    'norm_ind', 'batch_size', 'dataset', 'cond_set', 'static_spk', 'seed', 'weight_norm', 'qrnn',
    'scheduler', 'learning_rate'
]


def make_tag(params):
    """train.py:69-81: 'key:value' pairs of non-default tag params joined by '~'."""
    def to_string(v):
        if isinstance(v, bool):
            return 'T' if v else 'F'
        if isinstance(v, list):
            return ','.join(map(to_string, v))
        return str(v)
    return '~'.join(k + ':' + to_string(params[k]) for k in tag_params
                    if k not in default_params or params[k] != default_params[k])


def setup_results_dir(params):
    """train.py:84-103."""
    tag = make_tag(params)
    results_path = os.path.abspath(params['results_path'])
    os.makedirs(results_path, exist_ok=True)
    results_path = os.path.join(results_path, tag)
    if os.path.exists(results_path) and not params['resume']:
        shutil.rmtree(results_path)
    for sub in ('checkpoints', 'samples'):
        os.makedirs(os.path.join(results_path, sub), exist_ok=True)
    return results_path


def _ckpt_key(path):
    m = re.match(SaverPlugin.last_pattern.format(r'(\d+)', r'(\d+)'), os.path.basename(path))
    return (int(m.group(1)), int(m.group(2))) if m else (-1, -1)


def load_last_checkpoint(checkpoints_path):
    """train.py:106-121: newest ep{E}-it{I} (natural order) -> (state_dict, epoch, it)."""
    paths = sorted(glob(os.path.join(checkpoints_path, SaverPlugin.last_pattern.format('*', '*'))),
                   key=_ckpt_key)
    paths = [p for p in paths if _ckpt_key(p)[0] >= 0]
    if not paths:
        return None
    epoch, iteration = _ckpt_key(paths[-1])
    return torch.load(paths[-1], map_location='cpu', weights_only=True), epoch, iteration


def load_model(checkpoint_path):
    """train.py:152-166 / generate.py:72-86: state_dict + (epoch, iteration) from the name."""
    m = re.match('.*ep{}-it{}'.format(r'(\d+)', r'(\d+)'), os.path.basename(checkpoint_path))
    epoch, iteration = (int(m.group(1)), int(m.group(2))) if m else (0, 0)
    return torch.load(checkpoint_path, map_location='cpu', weights_only=True), epoch, iteration


def tee_stdout(log_path):
    """train.py:124-138."""
    log_file = open(log_path, 'a', 1)
    stdout = sys.stdout

    class Tee:
        def write(self, s):
            log_file.write(s)
            stdout.write(s)

        def flush(self):
            log_file.flush()
            stdout.flush()
    sys.stdout = Tee()


def init_random_seed(seed, cuda):
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if cuda:
        torch.cuda.manual_seed(seed)


class RowShard:
    """Iterates a full-batch loader and yields this rank's contiguous stream rows."""

    def __init__(self, loader, rows):
        self.loader, self.rows = loader, rows

    def __iter__(self):
        for data, reset, target, cond, spk in self.loader:
            r = self.rows
            yield data[r], reset[r] if torch.is_tensor(reset) else reset, target[r], cond[r], \
                spk[r]

    def __len__(self):
        return len(self.loader)


def make_data_loader(overlap_len, params, rows=None):
    """train.py:169-181 (FolderDataset + DataLoader(shuffle=False, drop_last=True))."""
    from torch.utils.data import DataLoader
    path = os.path.join(params['datasets_path'], params['dataset'])
    cond_path = os.path.join(params['cond_path'], params['cond_set'])

    def data_loader(partition):
        ds = FolderDataset(params['datasets_path'], path, cond_path, overlap_len,
                           params['q_levels'], params['ulaw'], params['seq_len'],
                           params['batch_size'], params['cond_dim'], params['cond_len'],
                           params['norm_ind'], params['static_spk'], params['look_ahead'],
                           partition)
        dl = DataLoader(ds, batch_size=params['batch_size'], shuffle=False, drop_last=True,
                        num_workers=2)
        return dl if rows is None else RowShard(dl, rows)
    return data_loader


def main(exp, frame_sizes, dataset, **params):
    dist_mod.init()
    use_cuda = torch.cuda.is_available()
    if use_cuda:
        torch.cuda.set_device(dist_mod.device_index())
    lead = dist_mod.rank() == 0
    params = dict(default_params, exp=exp, frame_sizes=frame_sizes, dataset=dataset, **params)
    init_random_seed(params['seed'], use_cuda)
    results_path = setup_results_dir(params)
    if lead:
        tee_stdout(os.path.join(results_path, 'log'))
    ds_dir = os.path.join(params['datasets_path'], params['dataset'])
    spk_dim = len([i for i in os.listdir(ds_dir) if os.path.islink(os.path.join(ds_dir, i))])
    model = SampleRNN(frame_sizes=params['frame_sizes'], n_rnn=params['n_rnn'],
                      dim=params['dim'], learn_h0=params['learn_h0'],
                      q_levels=params['q_levels'], ulaw=params['ulaw'],
                      weight_norm=params['weight_norm'],
                      cond_dim=params['cond_dim'] * (1 + params['look_ahead']),
                      spk_dim=spk_dim, qrnn=params['qrnn'])
    model.compute_dtype = torch.bfloat16 if params['compute_dtype'] == 'bf16' else torch.float32
    predictor = Predictor(model)
    if use_cuda:
        predictor = predictor.cuda()
    if params['model'] is not None:
        state_dict, _, _ = load_model(params['model'])
        predictor.load_state_dict(state_dict)
    optimizer = torch.optim.Adam(predictor.parameters(), lr=params['learning_rate'])
    scheduler = None
    if params['scheduler']:
        from torch.optim.lr_scheduler import MultiStepLR
        scheduler = MultiStepLR(optimizer, milestones=[15, 35], gamma=0.1)
    sync = dist_mod.GradAllReduce(overlap_groups=dist_mod.readiness_groups(predictor)) \
        if dist_mod.world() > 1 else None
    optimizer = gradient_clipping(optimizer, grad_sync=sync)
    rows = dist_mod.shard_rows(params['batch_size']) if dist_mod.world() > 1 else None
    data_loader = make_data_loader(model.lookback, params, rows)
    writer = None
    trainer = Trainer(predictor, sequence_nll_loss_bits, optimizer, data_loader('train'),
                      use_cuda, writer, scheduler)
    checkpoints_path = os.path.join(results_path, 'checkpoints')
    ck = load_last_checkpoint(checkpoints_path)
    if ck is not None:
        state_dict, trainer.epochs, trainer.iterations = ck
        predictor.load_state_dict(state_dict)
    trainer.register_plugin(TrainingLossMonitor(smoothing=params['loss_smoothing']))
    trainer.register_plugin(ValidationPlugin(data_loader('validation'), data_loader('test'),
                                             writer))
    trainer.register_plugin(AbsoluteTimeMonitor())
    if lead:
        trainer.register_plugin(SaverPlugin(checkpoints_path, params['keep_old_checkpoints']))
        trainer.register_plugin(Logger(['training_loss', 'validation_loss', 'test_loss', 'time']))
        trainer.register_plugin(StatsPlugin(
            results_path,
            iteration_fields=['training_loss', ('training_loss', 'running_avg'), 'time'],
            epoch_fields=['validation_loss', 'test_loss', 'time'],
            plots={'loss': {'x': 'iteration',
                            'ys': ['training_loss', ('training_loss', 'running_avg'),
                                   'validation_loss', 'test_loss'],
                            'log_y': True}}))
    trainer.run(params['epoch_limit'])


def parse_bool(arg):
    arg = arg.lower()
    if 'true'.startswith(arg):
        return True
    if 'false'.startswith(arg):
        return False
    raise ValueError(arg)


def build_parser():
    p = argparse.ArgumentParser(formatter_class=argparse.ArgumentDefaultsHelpFormatter,
                                argument_default=argparse.SUPPRESS)
    p.add_argument('--exp', required=True, help='experiment name')
    p.add_argument('--frame_sizes', nargs='+', type=int, required=True,
                   help='frame sizes in terms of the number of lower tier frames, '
                        'starting from the lowest RNN tier')
    p.add_argument('--dataset', required=True, help='dataset name (directory of WAV links)')
    p.add_argument('--cond_set', help='conditioning set name')
    for name, typ in (('n_rnn', int), ('dim', int), ('learn_h0', parse_bool),
                      ('ulaw', parse_bool), ('q_levels', int), ('seq_len', int),
                      ('batch_size', int), ('keep_old_checkpoints', parse_bool),
                      ('datasets_path', str), ('cond_path', str), ('results_path', str),
                      ('epoch_limit', int), ('resume', parse_bool), ('sample_rate', int),
                      ('n_samples', int), ('sample_length', int), ('loss_smoothing', float),
                      ('learning_rate', float), ('look_ahead', parse_bool), ('seed', int),
                      ('weight_norm', parse_bool), ('norm_ind', parse_bool),
                      ('static_spk', parse_bool), ('qrnn', parse_bool), ('model', str),
                      ('scheduler', parse_bool), ('compute_dtype', str)):
        p.add_argument('--' + name, type=typ)
    p.set_defaults(**default_params)
    return p


if __name__ == '__main__':
    main(**vars(build_parser().parse_args()))
