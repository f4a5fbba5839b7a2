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
file is O(runs) numpy slices instead of a Python loop over every frame.  The reference file
is MIT-licensed (c) 2016 Santi Dsp (interpolate.py:1-22); see THIRD_PARTY_NOTICES.md.
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


# unvoiced thresholds of the two Ahocoder streams (interpolate.py:97-105): log-F0 frames at
# or below -1e10, maximum-voiced-frequency frames at or below 1e3
THRESHOLDS = {'f0': -10000000000, 'vf': 1e3}


def _outputs(path):
    """(interpolation file, u/v file) next to `path`: <stem>.i<ext> and <stem>.uv."""
    folder, name = os.path.split(path.rstrip())
    stem, ext = os.path.splitext(name)
    return os.path.join(folder, stem + '.i' + ext), os.path.join(folder, stem + '.uv')


def process_file(filename, unvoiced_symbol, gen_uv):
    """interpolate.py:77-87: <stem>.i<ext> <- interpolated frames; with gen_uv the mask is
    announced as <stem>.uv but, as in the reference, written over the .i file."""
    interp_path, uv_path = _outputs(filename)
    interp, uv = interpolation(np.loadtxt(filename), unvoiced_symbol)
    print('Writing interpolation to {}'.format(interp_path))
    np.savetxt(interp_path, interp)
    if not gen_uv:
        return
    print('Writing u/v mask to {}'.format(uv_path))
    np.savetxt(interp_path, uv)             # the reference's destination (documented quirk)


def process_guia(guia_file, unvoiced_symbol, gen_uv):
    """interpolate.py:90-94: every path listed (one per line) in a guide file."""
    with open(guia_file) as fh:
        paths = [line.rstrip() for line in fh]
    for path in paths:
        process_file(path, unvoiced_symbol, gen_uv)


def main(opts):
    """interpolate.py:97-105: single files first, then guide files, f0 before vf."""
    jobs = ((opts.f0_file, process_file, 'f0'), (opts.f0_guia, process_guia, 'f0'),
            (opts.vf_file, process_file, 'vf'), (opts.vf_guia, process_guia, 'vf'))
    for target, run, stream in jobs:
        if target:
            run(target, THRESHOLDS[stream], opts.gen_uv)


def build_parser():
    """The reference's command line (interpolate.py:108-127): --f0_file / --f0_guia /
    --vf_file / --vf_guia and --no-uv."""
    p = argparse.ArgumentParser('Here are the main options to interpolate Ahocoder features')
    for stream, what in (('f0', 'lf0'), ('vf', 'vf')):
        p.add_argument('--%s_guia' % stream, type=str, default=None,
                       help='guide file listing the %s files to interpolate' % what)
        p.add_argument('--%s_file' % stream, type=str, default=None,
                       help='a single %s file to interpolate' % what)
    p.add_argument('--no-uv', dest='gen_uv', action='store_false',
                   help='do not generate the U/V masks')
    p.set_defaults(gen_uv=True)
    return p


if __name__ == '__main__':
    main(build_parser().parse_args())
