"""HBM traffic of one generation step from two rocprofv3 PMC passes over tools/gen_prof.py
(--pmc FETCH_SIZE, then --pmc WRITE_SIZE; separate runs, MI355X_MICROARCH.md HBM section):
every dispatch of the generation loop's kernels (the persistent sample loop, the tier ticks,
the per-launch bookkeeping), FETCH_SIZE kB x 2 (gfx950 tallies 128-B requests at 64 B) +
WRITE_SIZE kB, divided by the samples generated (16 per persistent launch).

  python tools/pmc_gen.py FETCH_DB WRITE_DB > profiles/r02_pmc_gen.txt
"""
import os
import sqlite3
import sys

LOOP = ('gen_mlp_kernel', 'skinny_kernel', 'gru_cell_ring_kernel', 'tier_input_tiled_kernel',
        'fold_gru_kernel',
        'advance_kernel', 'gen_noise_kernel')



def _csrc_hash():
    """samplernn_hip.csrc_hash(): the kernels these counters were taken on."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, 'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
    import samplernn_hip
    return samplernn_hip.csrc_hash()


def per_kernel(db, ctr):
    c = sqlite3.connect(db)
    rows = c.execute('select kernel_name, counter_name, value from counters_collection').fetchall()
    agg = {}
    for name, cn, v in rows:
        if cn != ctr:
            continue
        short = name.split('(')[0]
        if not any(k in short for k in LOOP):
            continue
        n, s = agg.get(short, (0, 0.0))
        agg[short] = (n + 1, s + v)
    return agg


def main(fdb, wdb, what='gen: tools/gen_prof.py bf16 20'):
    f = per_kernel(fdb, 'FETCH_SIZE')
    w = per_kernel(wdb, 'WRITE_SIZE')
    launches = sum(n for k, (n, _) in f.items() if 'gen_mlp_kernel' in k)
    steps = 16 * launches
    tot = 0.0
    print('# HBM traffic of the generation loop (B = 128, D = 1024), %s under rocprofv3 '
          '--pmc FETCH_SIZE / WRITE_SIZE' % what)
    print('# kernel  dispatches  FETCH kB x2  WRITE kB  (totals over the run)')
    for k in sorted(set(f) | set(w)):
        nf, sf = f.get(k, (0, 0.0))
        nw, sw = w.get(k, (0, 0.0))
        tot += 2 * sf + sw
        print('%-70s %6d %14.1f %12.1f' % (k[:70], nf, 2 * sf, sw))
    print('generation steps %d (16 per persistent launch, %d launches)' % (steps, launches))
    print('avg_step_bytes %d' % int(round(tot * 1024 / max(steps, 1))))
    print('csrc_hash %s' % _csrc_hash())


if __name__ == '__main__':
    main(*sys.argv[1:4])
