"""Per-kernel timeline of the last complete TBPTT step in a rocprofv3 --kernel-trace database
(steps delimited by the fused clip+Adam launch).  python tools/step_kernels.py DB [min_us]"""
import sqlite3
import sys

db = sys.argv[1]
min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
c = sqlite3.connect(db)
rows = c.execute('select name, start, end from kernels order by start').fetchall()
idx = [i for i, r in enumerate(rows) if r[0].startswith('adam_clip')]
a, b = idx[-2], idx[-1]
t0 = rows[a][2]
print('step span %.1f us, %d kernels' % ((rows[b][2] - rows[a][2]) / 1e3, b - a))
busy = 0.0
agg = {}
for name, s, e in rows[a + 1:b + 1]:
    d = (e - s) / 1e3
    busy += d
    short = name.split('(')[0][:70]
    agg[short] = agg.get(short, 0.0) + d
    if d >= min_us:
        print('%8.1f %7.1f  %s' % ((s - t0) / 1e3, d, short))
print('busy %.1f us' % busy)
for k, v in sorted(agg.items(), key=lambda kv: -kv[1])[:25]:
    print('%8.1f  %s' % (v, k))
