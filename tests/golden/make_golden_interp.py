"""Golden fixtures for interpolate.py by RUNNING THE REFERENCE's own
interpolate.py (numpy only; importable here).  Survey container only: /root/reference does
not exist on the GPU box.  Stores inputs and the reference's outputs in interp.npz.

Signals: Ahocoder-like log-F0 tracks (unvoiced = -1e10) and voicing-frequency tracks
(unvoiced <= 1e3) with leading / inner / trailing unvoiced runs, all-voiced, all-unvoiced,
single-frame runs and length-1/2 edge cases.

Usage:  python tests/golden/make_golden_interp.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = '/root/reference'


def signals(rng):
    out = []
    for n in (1, 2, 3, 7, 50, 400):
        for kind in ('lf0', 'vf'):
            for pat in range(6):
                v = rng.uniform(4.0, 6.0, n) if kind == 'lf0' else rng.uniform(1500, 7000, n)
                unv = -1e10 if kind == 'lf0' else rng.uniform(0, 1e3, n)
                mask = np.zeros(n, bool)
                if pat == 0:
                    mask = rng.random(n) < 0.3
                elif pat == 1:
                    mask[: n // 3] = True
                elif pat == 2:
                    mask[-(n // 3 or 1):] = True
                elif pat == 3:
                    mask[:] = True
                elif pat == 4:
                    mask = rng.random(n) < 0.7
                # pat 5: all voiced
                sig = np.where(mask, unv, v).astype(np.float64)
                out.append((kind, sig))
    return out


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import interpolate as ref
    rng = np.random.Generator(np.random.PCG64(2024))
    data = {}
    for i, (kind, sig) in enumerate(signals(rng)):
        sym = -10000000000 if kind == 'lf0' else 1e3
        isig, uv = ref.interpolation(sig, sym)
        data['sig_%d' % i] = sig
        data['sym_%d' % i] = np.float64(sym)
        data['isig_%d' % i] = isig
        data['uv_%d' % i] = uv
    data['n'] = np.int64(len(signals(np.random.Generator(np.random.PCG64(2024)))))
    np.savez_compressed(os.path.join(HERE, 'interp.npz'), **data)
    print('wrote interp.npz with', int(data['n']), 'signals')


if __name__ == '__main__':
    main()
