"""Drop-in for the reference's interpolate.py (interpolate.py:1-127): Ahocoder feature
interpolation over unvoiced frames.

Host-side feature preparation feeding dataset.py / generate.py: log-F0 frames are unvoiced
when <= -1e10, voicing-frequency frames when <= 1e3.  Same function names, arguments,
outputs and quirks as the reference:

  * a leading unvoiced run takes the first voiced value (uv = 0 there);
  * an inner unvoiced run is filled by a straight line from the LAST voiced frame before it
    (that frame included: it keeps its value but gets uv = 0) to the first voiced frame
    after it (excluded), values fb0 + k * ((fb1 - fb0) / n) in float64 (interpolate.py:40-44);
  * a trailing unvoiced run holds the last voiced value (from that frame on, uv = 0);
  * an all-unvoiced or all-voiced signal is returned unchanged with uv = 1 everywhere;
  * process_file writes the u/v mask over the interpolation file, not to `.uv`
    (interpolate.py:85-87; kept, documented).

The per-frame state machine is replaced by a run-length pass over the voiced mask, so a
file is O(runs) numpy slices instead of a Python loop over every frame.
"""
import argparse
import os

import numpy as np


def linear_interpolation(tbounds, fbounds):
    """interpolate.py:38-44: fbounds[0] + (t - t0) * ((f1 - f0) / (t1 - t0)), t in [t0, t1)."""
    t0, t1 = int(tbounds[0]), int(tbounds[1])
    f0, f1 = float(fbounds[0]), float(fbounds[1])
    slope = (f1 - f0) / (t1 - t0)
    return list(f0 + np.arange(t1 - t0, dtype=np.float64) * slope)


def interpolation(signal, unvoiced_symbol):
    """interpolate.py:47-74 -> (interpolated signal, uv mask int8)."""
    signal = np.asarray(signal)
    isignal = np.copy(signal)
    uv = np.ones(signal.shape, dtype=np.int8)
    n = signal.shape[0]
    if n < 2:
        return isignal, uv
    voiced = signal > unvoiced_symbol
    # transitions at t (1..n-1): onset = unvoiced(t-1) -> voiced(t), offset = voiced -> unvoiced
    prev, cur = voiced[:-1], voiced[1:]
    onsets = np.nonzero(~prev & cur)[0] + 1
    offsets = np.nonzero(prev & ~cur)[0] + 1
    oi = 0
    open_t0 = None              # last voiced frame before an open unvoiced run
    for t in onsets:
        # offsets before this onset: the first one opens the run (later ones cannot exist
        # without an onset in between)
        while oi < len(offsets) and offsets[oi] < t:
            if open_t0 is None:
                open_t0 = offsets[oi] - 1
            oi += 1
        if open_t0 is None:
            # leading unvoiced run (reference: tbound still [None, None])
            isignal[:t] = signal[t]
            uv[:t] = 0
        else:
            seg = linear_interpolation((open_t0, t), (signal[open_t0], signal[t]))
            isignal[open_t0:t] = seg
            uv[open_t0:t] = 0
            open_t0 = None
    if oi < len(offsets) and open_t0 is None:
        open_t0 = offsets[oi] - 1
    if open_t0 is not None:
        isignal[open_t0:] = signal[open_t0]
        uv[open_t0:] = 0
    return isignal, uv


def process_file(filename, unvoiced_symbol, gen_uv):
    """interpolate.py:77-87."""
    dire, fullname = os.path.split(filename.rstrip())
    basename, ext = os.path.splitext(fullname)
    raw = np.loadtxt(filename)
    interp, uv = interpolation(raw, unvoiced_symbol)
    out_interp_file = os.path.join(dire, basename + '.i' + ext)
    print('Writing interpolation to {}'.format(out_interp_file))
    np.savetxt(out_interp_file, interp)
    if gen_uv:
        out_uv_file = os.path.join(dire, basename + '.uv')
        print('Writing u/v mask to {}'.format(out_uv_file))
        np.savetxt(out_interp_file, uv)      # reference quirk: overwrites the .i file


def process_guia(guia_file, unvoiced_symbol, gen_uv):
    """interpolate.py:90-94."""
    with open(guia_file) as fh:
        for filename in fh:
            process_file(filename.rstrip(), unvoiced_symbol, gen_uv)


def main(opts):
    """interpolate.py:97-105."""
    if opts.f0_file:
        process_file(opts.f0_file, -10000000000, opts.gen_uv)
    if opts.f0_guia:
        process_guia(opts.f0_guia, -10000000000, opts.gen_uv)
    if opts.vf_file:
        process_file(opts.vf_file, 1e3, opts.gen_uv)
    if opts.vf_guia:
        process_guia(opts.vf_guia, 1e3, opts.gen_uv)


if __name__ == '__main__':
    parser = argparse.ArgumentParser('Here are the main options to interpolate Ahocoder features')
    parser.add_argument('--f0_guia', type=str, default=None,
                        help='Guia file containing pointers to the lf0 files to interpolate.')
    parser.add_argument('--f0_file', type=str, default=None, help='Filename of a single F0 file')
    parser.add_argument('--vf_guia', type=str, default=None,
                        help='Guia file containing pointers to the vf files to interpolate.')
    parser.add_argument('--vf_file', type=str, default=None, help='Filename of a single VF file')
    parser.add_argument('--no-uv', dest='gen_uv', action='store_false',
                        help='U/V masks are NOT generated.')
    parser.set_defaults(gen_uv=True)
    main(parser.parse_args())
