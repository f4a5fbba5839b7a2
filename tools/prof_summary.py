"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(float(r['TotalDurationNs']) for r in rows)
print('total kernel time %.3f ms' % (tot / 1e6))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:n]:
    print('%6.2f%% %9.3f ms calls=%6s avg=%9.1f us  %s' % (
        100 * float(r['TotalDurationNs']) / tot, float(r['TotalDurationNs']) / 1e6, r['Calls'],
        float(r['AverageNs']) / 1e3, r['Name'][:100]))
