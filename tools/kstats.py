"""Per-step kernel breakdown of a rocprofv3 --kernel-trace database (rocpd sqlite).

  python tools/kstats.py RUN_results.db FIRST LAST [--marker adam_clip_multi_kernel]

The steps are delimited by the marker kernel (one launch per TBPTT step: the fused clip +
Adam): the window runs from the end of marker launch FIRST-1 to the end of launch LAST
(0-based), i.e. steps FIRST..LAST.  Prints, per kernel name, launches / step, total and
mean duration, share of the window, plus the window's busy fraction (sum of kernel time /
wall time) -- the idle remainder is launch gaps.
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('db')
    ap.add_argument('first', type=int)
    ap.add_argument('last', type=int)
    ap.add_argument('--marker', default='adam_clip_multi_kernel')
    ap.add_argument('--sequence', action='store_true',
                    help='also list step FIRST kernel by kernel (start offset, duration)')
    ap.add_argument('--span', type=int, default=1, help='steps the sequence covers')
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute('select name, start, end from kernels order by start'))
    marks = [r for r in rows if a.marker in r[0]]
    t0 = marks[a.first - 1][2] if a.first > 0 else rows[0][1]
    t1 = marks[a.last][2]
    n = a.last - a.first + 1
    agg = {}
    busy = 0
    for name, s, e in rows:
        if s < t0 or e > t1:
            continue
        short = name.split('(')[0].replace('void ', '')[:90]
        d = agg.setdefault(short, [0, 0])
        d[0] += 1
        d[1] += e - s
        busy += e - s
    wall = t1 - t0
    print('steps %d..%d: %.3f ms/step wall, %.3f ms/step kernel time (busy %.1f %%)' % (
        a.first, a.last, wall / n / 1e6, busy / n / 1e6, 100.0 * busy / wall))
    print('%-90s %8s %10s %10s %6s' % ('kernel', 'per_step', 'ms/step', 'avg_us', 'share'))
    for k, (cnt, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print('%-90s %8.1f %10.4f %10.2f %5.1f%%' % (k, cnt / n, tot / n / 1e6, tot / cnt / 1e3,
                                                    100.0 * tot / wall))
    if a.sequence:
        s0 = marks[a.first - 1][2] if a.first > 0 else rows[0][1]
        s1 = marks[a.first + a.span - 1][2]
        print('\n# steps %d..%d in launch order: start offset us, duration us, kernel'
              % (a.first, a.first + a.span - 1))
        for name, s, e in rows:
            if s0 <= s and e <= s1:
                print('%9.1f %8.1f  %s' % ((s - s0) / 1e3, (e - s) / 1e3,
                                          name.split('(')[0].replace('void ', '')[:100]))


if __name__ == '__main__':
    main()
