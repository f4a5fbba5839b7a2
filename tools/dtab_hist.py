"""Sample-value histogram of the dTab scatter's index windows on the bench's synthetic
streams (bench.synth_batches: B = 512, T = 1024, chunk 0 and 1): what fraction of the
scatter's positions the most frequent 8 / 16 / 32 values cover -- the share a register
hot-bin cache could take off the LDS atomics.  CPU only:
python tools/dtab_hist.py"""
import os
import sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, '..'), os.path.join(HERE, '..', 'tests', 'golden'),
                os.path.join(HERE, '..', 'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd')]
import numpy as np  # noqa: E402
import bench  # noqa: E402

B, T, L, FS0 = 512, 1024, 64, 16
for n, (inp, _, _, _, _) in enumerate(bench.synth_batches(B, T, L, 2, 0)):
    win = inp[:, L - FS0:].numpy()            # the MLP's window: T + FS0 - 1 per row
    cnt = np.bincount(win.reshape(-1), minlength=256)
    s = np.sort(cnt)[::-1] / cnt.sum()
    print('chunk %d: %d positions, max count %d (value %d); top 8 / 16 / 32 values cover '
          '%.1f / %.1f / %.1f %% of positions' % (n, cnt.sum(), cnt.max(), cnt.argmax(),
                                                 100 * s[:8].sum(), 100 * s[:16].sum(),
                                                 100 * s[:32].sum()))
