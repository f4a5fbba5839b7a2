"""Per-step GPU timeline of a TBPTT profile (rocprofv3 --kernel-trace SQLite output): kernels per
step, span, busy time (union of kernel intervals) and the largest idle gaps between kernels --
whether the step is GPU-bound or waits on the host's launches.  Steps are delimited by the
fused clip+Adam launch that ends each one.

  python tools/step_timeline.py DB
"""
import sqlite3
import sys


def main(db):
    c = sqlite3.connect(db)
    rows = c.execute('select name, start, end from kernels order by start').fetchall()
    ends = [i for i, r in enumerate(rows) if r[0].startswith('adam_clip_multi')]
    print('%d kernels, %d steps' % (len(rows), len(ends)))
    for a, b in zip(ends[:-1], ends[1:]):
        seg = rows[a + 1:b + 1]
        span = (seg[-1][2] - seg[0][1]) / 1e3
        busy = 0
        cs, ce = seg[0][1], seg[0][2]
        for _, s, e in seg[1:]:
            if s > ce:
                busy += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        gaps = sorted(((seg[i + 1][1] - seg[i][2]) / 1e3, seg[i][0][:40], seg[i + 1][0][:40])
                      for i in range(len(seg) - 1))[::-1]
        print('step: %d kernels, span %.0f us, busy %.0f us, idle %.0f us' %
              (len(seg), span, busy / 1e3, span - busy / 1e3))
        for g in gaps[:6]:
            print('   gap %.1f us after %s before %s' % g)


if __name__ == '__main__':
    main(sys.argv[1])
