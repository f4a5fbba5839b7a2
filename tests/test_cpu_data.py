"""Host-side rows of SURVEY §8 f (CPU only): interpolate.py (pinned to the reference's own
outputs, tests/golden/interp.npz from make_golden_interp.py), FolderDataset's stream layout
(dataset.py; parity unpinned -- the reference module needs librosa, absent here -- checked
by the reference's documented invariants), the trainer plugins' log format (the regexes of
the reference's plotlog.py) and the compat shims.
"""
import os
import pickle
import re

import numpy as np
import pytest
import torch

from conftest import golden


def test_interpolation_matches_reference_golden():
    from interpolate import interpolation
    g = golden('interp')
    for i in range(int(g['n'])):
        isig, uv = interpolation(g['sig_%d' % i], float(g['sym_%d' % i]))
        assert uv.dtype == np.int8
        np.testing.assert_array_equal(uv, g['uv_%d' % i], err_msg='uv %d' % i)
        np.testing.assert_array_equal(isig, g['isig_%d' % i], err_msg='signal %d' % i)


def _write_corpus(root, files, seed=0, frames=(290, 310, 270, 330)):
    """wav/ (16-bit PCM) + cond/ (.cc 40 cols, .lf0 with -1e10 unvoiced, .gv with <=1e3) and
    the partition lists, the layout train.py / generate.py expect."""
    from scipy.io import wavfile
    rng = np.random.Generator(np.random.PCG64(seed))
    wav = os.path.join(root, 'wav')
    cond = os.path.join(root, 'cond')
    os.makedirs(wav, exist_ok=True)
    os.makedirs(cond, exist_ok=True)
    for j, name in enumerate(files):
        nfr = frames[j % len(frames)]
        n = nfr * 80 + int(rng.integers(0, 80))
        x = (rng.standard_normal(n) * 3000).clip(-32768, 32767).astype(np.int16)
        wavfile.write(os.path.join(wav, name + '.wav'), 16000, x)
        np.savetxt(os.path.join(cond, name + '.cc'), rng.standard_normal((nfr, 40)))
        lf0 = rng.uniform(4, 6, nfr)
        lf0[rng.random(nfr) < 0.3] = -1e10
        gv = rng.uniform(1500, 6000, nfr)
        gv[rng.random(nfr) < 0.3] = 0.0
        np.savetxt(os.path.join(cond, name + '.lf0'), lf0)
        np.savetxt(os.path.join(cond, name + '.gv'), gv)
    return wav + '/', cond + '/'


@pytest.fixture
def corpus(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    files = ['72a%03d' % i for i in range(3)] + ['75b%03d' % i for i in range(3)]
    wav, cond = _write_corpus(str(tmp_path), files)
    (tmp_path / 'wav_train.list').write_text('\n'.join(files) + '\n')
    return str(tmp_path) + '/', wav, cond, files


@pytest.mark.parametrize('norm_ind', [False, True])
def test_folder_dataset_layout(corpus, norm_ind):
    import utils
    from dataset import FolderDataset
    root, wav, cond, files = corpus
    B, seq_len, overlap, cond_len = 2, 320, 64, 80
    ds = FolderDataset(root, wav, cond, overlap, 256, True, seq_len, B, 43, cond_len, norm_ind,
                       False, False, 'train')
    names = ds.npy_names
    for k in ('data', 'cond', 'spk', 'audio', 'min_max', 'spk_id'):
        assert os.path.isfile(names[k]), k
    assert ds.data.shape[0] == B and ds.cond.shape[0] == B and ds.cond.shape[2] == 43
    # joint normalisation maps the train partition into [0, 1]
    if not norm_ind:
        assert ds.cond.min() >= -1e-12 and ds.cond.max() <= 1 + 1e-12
    assert len(ds) == ds.data.size // seq_len
    cpb = seq_len // cond_len
    # chunks whose input, target and conditioning windows lie inside the rows (the
    # reference's length counts a final partial chunk too)
    n_full = min((ds.data.shape[1] - overlap - seq_len) // seq_len + 1,
                 (ds.cond.shape[1] - 1 - cpb) // cpb + 1)
    assert n_full >= 3
    check = sorted({0, 1, 2, n_full - 1})
    n_batches = n_full
    for n in check:
        for r in range(B):
            data, reset, target, c, spk = ds[n * B + r]
            assert reset == (n == 0)
            assert data.shape == (overlap + seq_len - 1,) and target.shape == (seq_len,)
            # input and target are the same stream, target shifted by overlap_len
            assert torch.equal(data[overlap:], target[:-1])
            s0 = n * seq_len
            ref_in = utils.uquantize(torch.from_numpy(ds.data[r][s0:s0 + overlap + seq_len - 1]),
                                     256)
            assert torch.equal(data, ref_in)
            # conditioning: frames [n*S/80 + 1, ...) (the reference's +1 offset), float64
            f0 = n * (seq_len // cond_len) + 1
            assert c.dtype == torch.float64
            np.testing.assert_array_equal(c.numpy(), ds.cond[r][f0:f0 + seq_len // cond_len])
            frames = ds.global_spk[r][f0:f0 + seq_len // cond_len].astype(int)
            assert int(spk[0]) == int(np.argmax(np.bincount(frames)))
            # stateful layout: chunk n of row r continues chunk n-1 of row r
            if n > 0:
                prev = ds[(n - 1) * B + r][2]
                s_prev = (n - 1) * seq_len + overlap
                assert torch.equal(prev, utils.uquantize(
                    torch.from_numpy(ds.data[r][s_prev:s_prev + seq_len]), 256))
    # reload from the npy caches: identical items; look-ahead doubles cond with frame t+1
    ds2 = FolderDataset(root, wav, cond, overlap, 256, True, seq_len, B, 43, cond_len, norm_ind,
                        False, False, 'train')
    for i in [0, 1, B * n_batches - 1]:
        a, b = ds[i], ds2[i]
        assert torch.equal(a[0], b[0]) and torch.equal(a[3], b[3]) and torch.equal(a[4], b[4])
    ds3 = FolderDataset(root, wav, cond, overlap, 256, True, seq_len, B, 43, cond_len, norm_ind,
                        False, True, 'train')
    assert ds3.cond.shape[2] == 86
    np.testing.assert_array_equal(ds3.cond[:, :-1, 43:], ds3.cond[:, 1:, :43])
    np.testing.assert_array_equal(ds3.cond[:, -1, 43:], ds3.cond[:, -1, :43])
    assert os.path.isfile(names['cond'].replace('.npy', '_ahead.npy'))


def test_folder_dataset_alignment_rule(corpus):
    """dataset.py:99-110: files end on an 80-sample frame boundary (pad when oversize >= 60,
    else trim and drop the last conditioning frame)."""
    from dataset import FolderDataset, load_wav, read_conditioners
    root, wav, cond, files = corpus
    B = 1
    ds = FolderDataset(root, wav, cond, 64, 256, True, 160, B, 43, 80, False, False, False,
                       'train')
    total, frames = 0, 0
    for f in files:
        d, _ = load_wav(wav + f + '.wav')
        c = read_conditioners(cond + f)[0]
        over = d.shape[0] % 80
        n = d.shape[0] + (80 - over if over >= 60 else 0)
        nc = c.shape[0]
        if over <= 60 and over != 0:
            n -= over
            nc -= 1
        total += n
        frames += nc
    lon = 160 + 64
    num = B * (total // (B * lon * 80))
    assert ds.data.size == num * lon * 80
    assert ds.cond.shape[1] == (num * lon * 80) // 80


def test_load_wav_scaling(tmp_path):
    from scipy.io import wavfile
    from dataset import load_wav, write_wav
    x = np.array([-32768, -1, 0, 1, 32767], dtype=np.int16)
    wavfile.write(str(tmp_path / 'a.wav'), 16000, x)
    y, sr = load_wav(str(tmp_path / 'a.wav'))
    assert sr == 16000 and y.dtype == np.float32
    np.testing.assert_array_equal(y, x.astype(np.float32) / 32768)
    write_wav(str(tmp_path / 'b.wav'), y, 16000)
    z, _ = load_wav(str(tmp_path / 'b.wav'))
    np.testing.assert_array_equal(z, y)


class _FakeTrainer:
    def __init__(self):
        self.stats = {}
        self.iterations = 0


def test_logger_lines_match_plotlog_regexes(capsys):
    from trainer.plugins import AbsoluteTimeMonitor, Logger, TrainingLossMonitor
    tr = _FakeTrainer()
    mon = TrainingLossMonitor(smoothing=0.9)
    tm = AbsoluteTimeMonitor()
    log = Logger(['training_loss', 'validation_loss', 'test_loss', 'time'])
    for p in (mon, tm, log):
        p.register(tr)
    tr.stats.setdefault('validation_loss', {})['log_epoch_fields'] = ['{last:.4f}']
    tr.stats.setdefault('test_loss', {})['log_epoch_fields'] = ['{last:.4f}']
    losses = [8.0, 7.5, 7.25]
    for i, l in enumerate(losses, 1):
        tr.iterations = i
        mon.iteration(i, None, None, None, torch.tensor(l))
        tm.iteration(i)
        log.iteration(i)
    tr.stats['validation_loss']['last'] = 7.1
    tr.stats['test_loss']['last'] = 7.2
    mon.epoch(1)
    log.epoch(1)
    out = capsys.readouterr().out.splitlines()
    # plotlog.py:23-26
    iterpat = re.compile('training_loss:.*time:')
    trainpat = re.compile('training_loss: ([-0-9.]+)')
    valpat = re.compile('validation_loss: ([-0-9.]+)')
    testpat = re.compile('test_loss: ([-0-9.]+)')
    it_lines = [l for l in out if iterpat.search(l)]
    assert [float(trainpat.search(l).group(1)) for l in it_lines] == losses
    assert any(valpat.search(l) and float(valpat.search(l).group(1)) == 7.1 for l in out)
    assert any(testpat.search(l) and float(testpat.search(l).group(1)) == 7.2 for l in out)
    ra = 0.0
    for l in losses:
        ra = ra * 0.9 + l * 0.1
    assert abs(tr.stats['training_loss']['running_avg'] - ra) < 1e-12
    assert tr.stats['training_loss']['epoch_mean'] == sum(losses) / 3


def test_saver_and_stats_plugins(tmp_path):
    from trainer.plugins import SaverPlugin, StatsPlugin
    tr = _FakeTrainer()
    tr.model = torch.nn.Linear(2, 2)
    tr.iterations = 10
    sv = SaverPlugin(str(tmp_path), False)
    sv.register(tr)
    tr.stats['validation_loss'] = {'last': 3.0}
    sv.epoch(1)
    tr.iterations = 20
    tr.stats['validation_loss'] = {'last': 4.0}
    sv.epoch(2)
    names = sorted(os.listdir(tmp_path))
    assert names == ['best-ep1-it10', 'ep2-it20']
    sd = torch.load(str(tmp_path / 'ep2-it20'), weights_only=True)
    assert set(sd) == {'weight', 'bias'}
    st = StatsPlugin(str(tmp_path), ['training_loss'], ['validation_loss'], {})
    st.register(tr)
    tr.stats['training_loss'] = {'last': 1.5}
    st.iteration()
    st.epoch(1)
    with open(tmp_path / 'stats.pkl', 'rb') as f:       # written by this test itself
        data = pickle.load(f)
    assert data['iterations'][('training_loss', 'last')] == [1.5]
    assert data['epochs'][('validation_loss', 'last')] == [4.0]


def test_train_cli_tag_and_checkpoint_order(tmp_path):
    import train
    p = dict(train.default_params, exp='TEST', frame_sizes=[16, 4], dataset='wav/', dim=512,
             seed=1)
    assert train.make_tag(p) == 'exp:TEST~frame_sizes:16,4~dim:512~seed:1'
    ck = tmp_path / 'checkpoints'
    ck.mkdir()
    for e, it in ((2, 9), (10, 100), (9, 90)):
        torch.save({'x': torch.tensor([e])}, str(ck / ('ep%d-it%d' % (e, it))))
    sd, e, it = train.load_last_checkpoint(str(ck))
    assert (e, it) == (10, 100) and int(sd['x']) == 10


def test_generate_cli_name_and_tag_parse():
    import generate
    assert generate.output_name('results/exp:A~dim:512/checkpoints/best-ep3-it7', 'T6B7', '72') \
        == 'results/exp:A~dim:512/samples/best-ep3-it7_file-T6B7_spk-72.wav'
    assert generate.as_type('T', bool) is True and generate.as_type('16,4', list) == [16, 4]


def test_compat_shims_install():
    import sys
    import compat
    compat.install()
    from torch.utils.trainer.plugins import Logger, LossMonitor  # noqa: F401
    from torch.utils.trainer.plugins.plugin import Plugin  # noqa: F401
    import natsort
    assert natsort.natsorted(['ep10-it1', 'ep9-it1', 'ep2-it3']) == ['ep2-it3', 'ep9-it1',
                                                                       'ep10-it1']
    assert 'librosa.output' in sys.modules and 'tensorboardX' in sys.modules
