"""Per-(kernel, grid) time per step from a rocprofv3 kernel_trace.csv.
usage: trace_summary.py run_kernel_trace.csv STEPS [N]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 40
agg = collections.defaultdict(list)
for r in rows:
    key = (r['Kernel_Name'][:70], r['Grid_Size_X'], r['Grid_Size_Y'], r['Grid_Size_Z'])
    agg[key].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
tot = sum(sum(v) for v in agg.values())
print('total %.3f ms/step over %d kernels' % (tot / steps / 1e6, len(rows)))
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:n]:
    print('%7.3f ms/step n/step=%6.1f avg=%8.1f us  %s grid=%s,%s,%s' % (
        sum(v) / steps / 1e6, len(v) / steps, sum(v) / len(v) / 1e3, k[0], k[1], k[2], k[3]))
