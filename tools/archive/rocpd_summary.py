"""Summarise a rocprofv3 SQLite output (run_results.db, the ROCm 7.x default format).

  python tools/archive/rocpd_summary.py stats DB [N]          -> kernel_stats CSV (rocprofv3 --stats form)
  python tools/archive/rocpd_summary.py pmc DB NAME_SUBSTR    -> per-dispatch counter values of matching
                                                         kernels + their average (kB for *_SIZE)
"""
import csv
import sqlite3
import statistics
import sys


def stats(db, n=None, out=sys.stdout):
    c = sqlite3.connect(db)
    rows = c.execute('select name, duration from kernels').fetchall()
    agg = {}
    for name, d in rows:
        agg.setdefault(name, []).append(d)
    tot = sum(sum(v) for v in agg.values())
    w = csv.writer(out, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(['Name', 'Calls', 'TotalDurationNs', 'AverageNs', 'Percentage', 'MinNs', 'MaxNs',
                'StdDev'])
    items = sorted(agg.items(), key=lambda kv: -sum(kv[1]))
    for name, v in items[:n]:
        s = sum(v)
        w.writerow([name, len(v), s, s / len(v), 100.0 * s / tot, min(v), max(v),
                    statistics.pstdev(v) if len(v) > 1 else 0.0])


def pmc(db, sub):
    c = sqlite3.connect(db)
    rows = c.execute('select dispatch_id, kernel_name, counter_name, value, duration from '
                     'counters_collection').fetchall()
    hit = [r for r in rows if sub in r[1]]
    by = {}
    for d, name, ctr, v, dur in hit:
        by.setdefault(ctr, []).append(v)
        print('%6d %-12s %14.1f %s' % (d, ctr, v, name[:80]))
    for ctr, v in by.items():
        print('avg %s over %d dispatches: %.1f' % (ctr, len(v), sum(v) / len(v)))


if __name__ == '__main__':
    if sys.argv[1] == 'stats':
        stats(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else None)
    elif sys.argv[1] == 'pmc':
        pmc(sys.argv[2], sys.argv[3])
