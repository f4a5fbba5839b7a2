"""Drop-in for the reference's dataset.py (dataset.py:1-292): FolderDataset, the stateful
TBPTT data layout that makes row-sharded data parallelism correct.

Same class name, constructor signature, npy cache files (names, contents, shapes), stream
layout and __getitem__ tuple `(data, reset, target, cond, spk)` as the reference, so a
DataLoader(batch_size=B, shuffle=False) over it yields the reference's batches:

  * the concatenated corpus is cut into `batch_size` continuous streams (rows); item
    index = n_batch * batch_size + row; chunk n of row r is input samples
    [n*seq_len, n*seq_len + overlap_len + seq_len - 1), target [overlap_len + n*seq_len, ..)
    (dataset.py:242-254), so consecutive batches continue each row's stream and the
    hidden state carried by Runner stays valid;
  * reset is True only for n_batch == 0 (dataset.py:261-266);
  * conditioning frames [n*seq_len/cond_len + 1, ... + seq_len/cond_len) -- the `+ 1`
    frame offset of the reference (dataset.py:263-266), float64;
  * speaker = the majority speaker id over those frames (dataset.py:280);
  * mu-law quantisation per item in float64 (dataset.py:253-254) through utils.uquantize,
    which is bit-exact to the reference for every input.

Creation path (dataset.py:58-209) kept, including its quirks: the 80-sample alignment with
the `oversize` rule (dataset.py:99-110, the two branches both run at oversize == 60),
per-speaker or joint min-max normalisation computed on the train partition and cached in
npy_datasets/min_max_{ind,joint}[_static].npy, and look-ahead conditioning applied only
when an existing dataset is LOADED (cached as *_ahead.npy, dataset.py:213-221).  librosa
is replaced by scipy.io.wavfile with librosa's int -> float scaling (x / 2^(bits-1),
float32, channels averaged).
"""
import os

import numpy as np
import torch
from torch.utils.data import Dataset

import utils
from interpolate import interpolation


def load_wav(path):
    """librosa.core.load(path, sr=None, mono=True)[0] for PCM/float WAV files: float32 in
    [-1, 1), int samples scaled by 1 / 2^(bits-1) (librosa.util.buf_to_float), channels
    averaged."""
    from scipy.io import wavfile
    sr, x = wavfile.read(path)
    if x.dtype == np.uint8:
        y = (x.astype(np.float32) - 128.0) * np.float32(1.0 / 128)
    elif np.issubdtype(x.dtype, np.integer):
        y = x.astype(np.float32) * np.float32(1.0 / float(1 << (8 * x.dtype.itemsize - 1)))
    else:
        y = x.astype(np.float32)
    if y.ndim == 2:
        y = np.mean(y, axis=1, dtype=np.float32)
    return y, sr


def write_wav(path, y, sr, norm=False):
    """librosa.output.write_wav (0.6): float32 WAV, optionally peak-normalised."""
    from scipy.io import wavfile
    y = np.asarray(y, dtype=np.float32)
    if norm and np.abs(y).max() > 0:
        y = y / np.abs(y).max()
    wavfile.write(path, int(sr), y)


def _npy_names(partition, norm_ind, static_spk):
    st = '_static' if static_spk else ''
    nrm = '_ind' if norm_ind else '_joint'
    base = 'npy_datasets/' + partition + '/'
    return {
        'data': base + 'data' + st + '.npy',
        'spk': base + 'speakers' + st + '.npy',
        'audio': base + 'audio_id' + st + '.npy',
        'min_max': 'npy_datasets/min_max' + nrm + st + '.npy',
        'cond': base + 'conditioners' + nrm + st + '.npy',
        'spk_id': 'npy_datasets/spk_id' + st + '.npy',
    }


def read_conditioners(stem):
    """One file's Ahocoder conditioning (dataset.py:85-96, generate.py:148-166):
    [cc (40) | interpolated lf0 | interpolated fv | u/v of fv] per 80-sample frame."""
    c = np.loadtxt(stem + '.cc')
    c = c.reshape(-1, c.shape[1])
    f0, _ = interpolation(np.loadtxt(stem + '.lf0'), -10000000000)
    fv, uv = interpolation(np.loadtxt(stem + '.gv'), 1e3)
    n = fv.shape[0]
    return c, f0.reshape(f0.shape[0], 1), fv.reshape(n, 1), uv.reshape(n, 1)


class FolderDataset(Dataset):
    """dataset.py:13-292."""

    def __init__(self, datasets_path, path, cond_path, overlap_len, q_levels, ulaw, seq_len,
                 batch_size, cond_dim, cond_len, norm_ind, static_spk, look_ahead, partition):
        super().__init__()
        self.overlap_len = overlap_len
        self.q_levels = q_levels
        self.ulaw = ulaw
        self.quantize = utils.uquantize if ulaw else utils.linear_quantize
        self.seq_len = seq_len
        self.batch_size = batch_size
        self.cond_dim = cond_dim
        self.cond_len = cond_len
        names = _npy_names(partition, norm_ind, static_spk)
        self.npy_names = names
        need = [names['data'], names['cond'], names['spk'], names['min_max']]
        if not all(os.path.isfile(f) for f in need):
            self._create(datasets_path, path, cond_path, norm_ind, static_spk, partition, names)
        else:
            self.data = np.load(names['data'])
            self.global_spk = np.load(names['spk'])
            if look_ahead:
                ahead = names['cond'].replace('.npy', '_ahead.npy')
                if os.path.isfile(ahead):
                    self.cond = np.load(ahead)
                else:
                    cond = np.load(names['cond'])
                    nxt = np.copy(cond)
                    nxt[:, :-1, :] = nxt[:, 1:, :]          # frame t+1; the last frame repeats
                    self.cond = np.concatenate((cond, nxt), axis=2)
                    np.save(ahead, self.cond)
            else:
                self.cond = np.load(names['cond'])
            mm = np.load(names['min_max'])
            self.min_cond, self.max_cond = mm[0], mm[1]
            self.length = int(np.prod(self.data.shape)) // self.seq_len
            print('Data shape:', self.data.shape)
            print('Conditioners shape:', self.cond.shape)
            print('Global speaker shape:', self.global_spk.shape)
            print('Dataset loaded for ' + partition + ' partition', '-' * 60, '\n')

    # ---------------------------------------------------------------- creation
    def _create(self, datasets_path, path, cond_path, norm_ind, static_spk, partition, names):
        st = '_static' if static_spk else ''
        print('Create ' + partition + ' dataset', '-' * 60, '\n')
        file_names = open(datasets_path + 'wav_' + partition + st + '.list').read().splitlines()
        for d in (os.path.dirname(names['data']), os.path.dirname(names['spk_id'])):
            if d:
                os.makedirs(d, exist_ok=True)
        if not os.path.isfile(names['spk_id']):
            spk = np.asarray(sorted({f[0:2] for f in file_names}))
            np.save(names['spk_id'], spk)
        else:
            spk = np.load(names['spk_id'])
        datas, conds, spks, audios = [], [], [], []
        for counter, name in enumerate(file_names):
            d, _ = load_wav(path + name + '.wav')     # float32; float64 once padded / appended
            c, f0, fv, uv = read_conditioners(cond_path + name)
            n = fv.shape[0]
            speaker = np.repeat(np.where(spk == name[0:2])[0][0], n)
            audio = np.repeat(counter, n)
            oversize = d.shape[0] % 80                # dataset.py:99-110 ('nosync')
            if oversize >= 60:
                d = np.append(d, np.zeros(80 - oversize))
            if oversize <= 60 and oversize != 0:
                d = d[:-oversize]
                c, f0, fv, uv = c[:-1], f0[:-1], fv[:-1], uv[:-1]
            if not self.ulaw:
                d = self.quantize(torch.from_numpy(d), self.q_levels).numpy()
            datas.append(d)
            conds.append(np.concatenate((c, f0, fv, uv), axis=1))
            spks.append(speaker.astype(np.float64))
            audios.append(audio.astype(np.float64))
        data = np.concatenate([x.astype(np.float64) for x in datas]) if datas else np.zeros(0)
        cond = np.concatenate(conds, axis=0) if conds else np.zeros((0, self.cond_dim))
        gspk = np.concatenate(spks) if spks else np.zeros(0)
        audio = np.concatenate(audios) if audios else np.zeros(0)
        total = data.shape[0]
        dim_cond = cond.shape[1]
        lon_seq = self.seq_len + self.overlap_len
        self.num_samples = self.batch_size * (total // (self.batch_size * lon_seq * self.cond_len))
        self.total_samples = self.num_samples * lon_seq * self.cond_len
        n_cond = self.total_samples // self.cond_len
        B = self.batch_size
        self.data = data[:self.total_samples].reshape(B, -1)
        self.length = self.total_samples // self.seq_len
        self.cond = cond[:n_cond].reshape(B, -1, dim_cond)
        self.global_spk = gspk[:n_cond].reshape(B, -1)
        self.audio = audio[:n_cond].reshape(B, -1)
        if partition == 'train' and not os.path.isfile(names['min_max']):
            if norm_ind:
                self.max_cond = np.empty((len(spk), self.cond_dim))
                self.min_cond = np.empty((len(spk), self.cond_dim))
                for i in range(len(spk)):
                    sel = self.cond[self.global_spk == i]
                    self.max_cond[i] = np.amax(sel, axis=0)
                    self.min_cond[i] = np.amin(sel, axis=0)
            else:
                self.max_cond = np.amax(np.amax(self.cond, axis=1), axis=0)
                self.min_cond = np.amin(np.amin(self.cond, axis=1), axis=0)
            np.save(names['min_max'], np.array([self.min_cond, self.max_cond]))
        else:
            mm = np.load(names['min_max'])
            self.min_cond, self.max_cond = mm[0], mm[1]
        if norm_ind:
            for i in range(len(spk)):
                sel = self.global_spk == i
                self.cond[sel] = (self.cond[sel] - self.min_cond[i]) / \
                                 (self.max_cond[i] - self.min_cond[i])
        else:
            self.cond = (self.cond - self.min_cond) / (self.max_cond - self.min_cond)
        np.save(names['data'], self.data)
        np.save(names['cond'], self.cond)
        np.save(names['spk'], self.global_spk)
        np.save(names['audio'], self.audio)
        print('Dataset created for ' + partition + ' partition', '-' * 60, '\n')

    # ---------------------------------------------------------------- items
    def __getitem__(self, index):
        n_batch, row = divmod(index, self.batch_size)
        start_data = n_batch * self.seq_len
        start_target = start_data + self.overlap_len
        end_target = start_target + self.seq_len
        stream = self.data[row]
        if not self.ulaw:
            data = torch.from_numpy(stream[start_data:end_target - 1]).long()
            target = torch.from_numpy(stream[start_target:end_target]).long()
        else:
            data = self.quantize(torch.from_numpy(stream[start_data:end_target - 1]), self.q_levels)
            target = self.quantize(torch.from_numpy(stream[start_target:end_target]), self.q_levels)
        cond_in_seq = self.seq_len // self.cond_len
        reset = n_batch == 0
        from_cond = n_batch * cond_in_seq + 1
        to_cond = from_cond + cond_in_seq
        cond = torch.from_numpy(self.cond[row][from_cond:to_cond])
        spk_frames = self.global_spk[row][from_cond:to_cond]
        spk = torch.from_numpy(np.array([np.argmax(np.bincount(spk_frames.astype(int)))]))
        return data, reset, target, cond, spk

    def __len__(self):
        return self.length
