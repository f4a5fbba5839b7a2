"""Drop-in for the reference's generate.py (generate.py:1-346): the generation CLI that
gen.sh calls (gen.sh:56), on the device generation path.

Same arguments and defaults, the experiment-tag re-parse of --model's directory
(generate.py:122-126: 'key:value~key:value' overrides), the conditioning pipeline
(.cc + interpolated .lf0 / .gv + u/v, min-max normalisation from
npy_datasets/min_max_{ind,joint}[_static].npy, optional look-ahead), the per-file seed, the
spk_dim rule (number of symlinks in datasets_path/cond_set) and the output file name
`<results>/<tag>/samples/<ckpt>_file-<name>_spk-<id>.wav` (float32, sample_rate).

Two sampling modes:
  * --sampler torch (default): the reference's behaviour file by file -- reseed, build the
    model (same RNG consumption as the reference's init), draw Exp(1) noise from torch's CPU
    generator in the reference's order: the sample stream replays the reference's.
  * --sampler philox --batch_files true: every file of the list in ONE device call (rows =
    files x n_samples, conditioning zero-padded to the longest file, outputs trimmed to each
    file's own length -- rows never interact), noise from the on-device Philox generator.
"""
import argparse
import os
import random
import re
import sys

import numpy as np
import torch

from dataset import read_conditioners, write_wav
from model import Generator, Predictor, SampleRNN, shard_generate

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
    'val_frac': 0.1,
    'test_frac': 0.1,
    'cond_dim': 43,
    'norm_ind': False,
    'static_spk': False,
    # training parameters
    'sample_rate': 16000,
    'n_samples': 1,
    'sample_length': 80000,
    'seed': 77977,
    'cond': 0,
    # generator parameters
    'datasets_path': '/veu/tfgveu7/project/tcstar/',
    'cond_set': 'cond/',
    'cond_list': 'generate_cond_gina.list',
    'spk_list': 'generate_spk_gina.list',
    'sampler': 'torch',
    'batch_files': False,
    'compute_dtype': 'fp32',
}


def init_random_seed(seed, cuda):
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if cuda:
        torch.cuda.manual_seed(seed)


def as_type(var, target_type):
    """generate.py:53-64: re-type a tag value like the default it overrides."""
    if target_type is bool:
        return var[0] == 'T'
    if target_type is int:
        return int(var)
    if target_type is float:
        return float(var)
    if target_type is list:
        return list(map(int, var.split(',')))
    return var


def load_model(checkpoint_path):
    """generate.py:67-84."""
    m = re.match('.*ep{}-it{}'.format(r'(\d+)', r'(\d+)'), os.path.basename(checkpoint_path))
    epoch, iteration = (int(m.group(1)), int(m.group(2))) if m else (0, 0)
    return torch.load(checkpoint_path, map_location='cpu', weights_only=True), epoch, iteration


def output_name(checkpoints_path, original_name, spk_name):
    """generate.py:99-101."""
    parts = checkpoints_path.split('/')
    return '/'.join(parts[:2]) + '/samples/' + parts[-1] + '_file-' + original_name + \
        '_spk-' + spk_name + '.wav'


def file_conditioning(stem, speaker, params):
    """generate.py:146-185: [cc | lf0 | fv | uv], normalised, optional look-ahead."""
    c, f0, fv, uv = read_conditioners(stem)
    cond = np.concatenate((c, f0, fv, uv), axis=1)
    st = '_static' if params['static_spk'] else ''
    mm = np.load('npy_datasets/min_max' + ('_ind' if params['norm_ind'] else '_joint') + st +
                 '.npy')
    lo, hi = mm[0], mm[1]
    if params['norm_ind']:
        cond = (cond - lo[speaker]) / (hi[speaker] - lo[speaker])
    else:
        cond = (cond - lo) / (hi - lo)
    if params['look_ahead']:
        nxt = np.copy(cond)
        nxt[:-1, :] = nxt[1:, :]
        cond = np.concatenate((cond, nxt), axis=1)
    return cond


def build_model(params, spk_dim, use_cuda):
    model = SampleRNN(frame_sizes=params['frame_sizes'], n_rnn=params['n_rnn'],
                      dim=params['dim'], learn_h0=params['learn_h0'],
                      q_levels=params['q_levels'], ulaw=params['ulaw'],
                      weight_norm=params['weight_norm'],
                      cond_dim=params['cond_dim'] * (1 + params['look_ahead']),
                      spk_dim=spk_dim, qrnn=params['qrnn'])
    model.compute_dtype = torch.bfloat16 if params['compute_dtype'] == 'bf16' else torch.float32
    predictor = Predictor(model)
    if use_cuda:
        model = model.cuda()
        predictor = predictor.cuda()
    state_dict, _, _ = load_model(params['model'])
    predictor.load_state_dict(state_dict)
    return model


def main(frame_sizes, **params):
    import distributed as Dd
    Dd.init()                   # torchrun: one process per GPU (no-op for a single process)
    use_cuda = torch.cuda.is_available()
    if use_cuda:
        torch.cuda.set_device(Dd.device_index())
    rank, world = Dd.rank(), Dd.world()
    params = dict(default_params, frame_sizes=frame_sizes, **params)
    # parameters encoded in the experiment directory name (generate.py:122-126)
    parts = params['model'].split('/')
    if len(parts) > 1:
        for item in parts[1].split('~'):
            kv = item.split(':')
            if len(kv) == 2 and kv[0] in params:
                params[kv[0]] = as_type(kv[1], type(params[kv[0]]))
    root = str(params['datasets_path'])
    file_names = open(root + params['cond_list']).read().splitlines()
    spk_names = open(root + params['spk_list']).read().splitlines()
    if len(spk_names) != len(file_names):
        sys.exit('Length of speaker file do not match length of conditioner file.')
    cond_dir = os.path.join(root, params['cond_set'])
    spk = np.load('npy_datasets/spk_id.npy')
    spk_dim = len([i for i in os.listdir(cond_dir) if os.path.islink(os.path.join(cond_dir, i))])
    jobs = []
    for name, spk_name in zip(file_names, spk_names):
        speaker = int(np.where(spk == spk_name)[0][0])
        original = name.split('/')[1] if '/' in name else name
        if original == '..':
            original = name.split('/')[3]
        jobs.append((cond_dir + name, speaker, original))
    if params['batch_files']:
        init_random_seed(params['seed'], use_cuda)
        model = build_model(params, spk_dim, use_cuda)
        conds = [file_conditioning(stem, sp, params) for stem, sp, _ in jobs]
        n = params['n_samples']
        n_cond = max(c.shape[0] for c in conds)
        C = conds[0].shape[1]
        rows = np.zeros((len(jobs) * n, n_cond, C), dtype=np.float32)
        spks = np.zeros(len(jobs) * n, dtype=np.int64)
        for j, c in enumerate(conds):
            rows[j * n:(j + 1) * n, :c.shape[0]] = c
            spks[j * n:(j + 1) * n] = jobs[j][1]
        gen = Generator(model, use_cuda)
        if world > 1:
            # rank-sharded: contiguous row shards gathered at the end (rows
            # padded to a multiple of the world size); either sampler reproduces the
            # single-process stream (shard_generate)
            pad = (-len(rows)) % world
            prow = np.concatenate([rows, np.zeros((pad,) + rows.shape[1:], rows.dtype)])
            pspk = np.concatenate([spks, np.zeros(pad, spks.dtype)])
            out = shard_generate(gen, len(prow), prow, pspk, params['seed'],
                                 sampler=params['sampler'], noise_rows=len(rows),
                                 seq_len=params['sample_length']).numpy()[:len(rows)]
        else:
            out = gen(len(rows), params['sample_length'], rows, spks, sampler=params['sampler'],
                      seed=params['seed']).numpy()
        if rank != 0:
            return
        L = model.lookback
        for j, (stem, sp, original) in enumerate(jobs):
            fname = output_name(params['model'], original, str(spk[sp]))
            for i in range(n):
                write_wav(fname, out[j * n + i, :conds[j].shape[0] * L], sr=params['sample_rate'])
        return
    for j, (stem, speaker, original) in enumerate(jobs):
        if j % world != rank:       # files are independent: round-robin over the ranks
            continue
        cond = file_conditioning(stem, speaker, params)
        init_random_seed(params['seed'], use_cuda)
        model = build_model(params, spk_dim, use_cuda)
        fname = output_name(params['model'], original, str(spk[speaker]))
        print('Generating file', fname)
        gen = Generator(model, use_cuda)
        samples = gen(params['n_samples'], params['sample_length'], cond, speaker,
                      sampler=params['sampler'], seed=params['seed']).numpy()
        for i in range(params['n_samples']):
            write_wav(fname, samples[i, :], sr=params['sample_rate'])


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
    p.add_argument('--frame_sizes', nargs='+', type=int, required=True,
                   help='frame sizes in terms of the number of lower tier frames, '
                        'starting from the lowest RNN tier')
    p.add_argument('--model', required=True, help='model (including path)')
    for name, typ in (('n_rnn', int), ('dim', int), ('learn_h0', parse_bool),
                      ('ulaw', parse_bool), ('q_levels', int), ('seq_len', int),
                      ('batch_size', int), ('datasets_path', str), ('cond_set', str),
                      ('sample_rate', int), ('n_samples', int), ('sample_length', int),
                      ('norm_ind', parse_bool), ('look_ahead', float),
                      ('static_spk', parse_bool), ('seed', int), ('weight_norm', parse_bool),
                      ('cond_list', str), ('spk_list', str), ('sampler', str),
                      ('batch_files', parse_bool), ('compute_dtype', str)):
        p.add_argument('--' + name, type=typ)
    # gen.sh passes --results_path (generate.py has no such option; accepted and ignored)
    p.add_argument('--results_path', type=str)
    p.set_defaults(**default_params)
    return p


if __name__ == '__main__':
    args = vars(build_parser().parse_args())
    args.pop('results_path', None)
    if isinstance(args.get('look_ahead'), float):
        args['look_ahead'] = bool(args['look_ahead'])
    main(**args)
