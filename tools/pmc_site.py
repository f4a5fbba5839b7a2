"""HBM traffic per TBPTT step of one probed launch site from two rocprofv3 PMC passes over
bench.py (--pmc FETCH_SIZE, then --pmc WRITE_SIZE; separate runs, MI355X_MICROARCH.md HBM
section): the site's kernels, mean per dispatch of FETCH_SIZE kB x 2 (gfx950 tallies 128-B
requests at 64 B) + WRITE_SIZE kB, summed over the kernels the site launches once per step.

  python tools/pmc_site.py SITE ROWS FETCH_DB WRITE_DB kernel1 [kernel2 ...]
      > profiles/r03_pmc_<SITE>_b<ROWS>.txt      (read back by bench.py pmc_traffic)
"""
import os
import sqlite3
import sys



def _csrc_hash():
    """samplernn_hip.csrc_hash(): the kernels these counters were taken on."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, 'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
    import samplernn_hip
    return samplernn_hip.csrc_hash()


def per_kernel(db, ctr, names):
    c = sqlite3.connect(db)
    rows = c.execute('select kernel_name, counter_name, value from counters_collection').fetchall()
    agg = {}
    for name, cn, v in rows:
        if cn != ctr:
            continue
        short = name.split('(')[0].replace(' ', '')     # template names: given without spaces
        key = next((k for k in names if k in short), None)
        if key is None:
            continue
        n, s = agg.get(key, (0, 0.0))
        agg[key] = (n + 1, s + v)
    return agg


def main(site, rows, fdb, wdb, names):
    f = per_kernel(fdb, 'FETCH_SIZE', names)
    w = per_kernel(wdb, 'WRITE_SIZE', names)
    print('# HBM traffic of the %s site per TBPTT step (bf16, %s rows, D = 1024), bench.py under '
          'rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate runs)' % (site, rows))
    print('# kernel  dispatches  mean FETCH kB x2  mean WRITE kB  (per dispatch)')
    tot = 0.0
    for k in names:
        nf, sf = f.get(k, (0, 0.0))
        nw, sw = w.get(k, (0, 0.0))
        mf = 2 * sf / nf if nf else 0.0
        mw = sw / nw if nw else 0.0
        tot += mf + mw
        print('%-40s %6d %14.1f %12.1f' % (k, nf, mf, mw))
    print('avg_step_bytes %d' % int(round(tot * 1024)))
    print('csrc_hash %s' % _csrc_hash())


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4], sys.argv[5:])
