#!/bin/bash
# LDS-side counters of the L1 gather and the dTab scatter (one rocprofv3 --pmc pass of SQ
# counters over a short B = 512 bench run): which of the wanted counters this ROCm lists, then
# one pass with them, summarised per kernel -> gpurun_out/<TAG>_pmc_lds.txt
set -e
R=$PWD; O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
TAG=${TAG:-r05}
timeout -s KILL 60 rocprofv3 -L > $O/${TAG}_rocprof_list.txt 2>&1 || true
CTRS=$(python3 - "$O/${TAG}_rocprof_list.txt" <<'PY'
import sys, re
txt = open(sys.argv[1]).read()
want = ['SQ_INSTS_LDS', 'SQ_LDS_BANK_CONFLICT', 'SQ_LDS_ADDR_CONFLICT', 'SQ_WAIT_INST_LDS',
        'SQ_INSTS_VALU', 'SQ_WAVE_CYCLES', 'SQ_BUSY_CYCLES', 'SQ_ACTIVE_INST_LDS']
have = [c for c in want if re.search(r'\b%s\b' % c, txt)]
print(' '.join(have[:8]))
PY
)
echo "counters: $CTRS"
rm -rf /tmp/plds
timeout -s KILL 120 rocprofv3 --pmc $CTRS -d /tmp/plds -o run -- python3 $R/bench.py --steps 2 --warmup 2 --no-gen --no-cpu --no-extra --batch 512 > $O/${TAG}_pmc_lds_run.log 2>&1
python3 - $(find /tmp/plds -name '*.db' | head -1) > $O/${TAG}_pmc_lds.txt <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
rows = c.execute('select kernel_name, counter_name, value from counters_collection').fetchall()
agg = {}
for name, cn, v in rows:
    short = name.split('(')[0]
    for key in ('mlp_l1_lds_kernel', 'dtab_pk_kernel', 'gemm3p_kernel<__hip_bfloat16, true, true, true, 2'):
        if key in short:
            n, s = agg.get((key, cn), (0, 0.0))
            agg[(key, cn)] = (n + 1, s + v)
print('# per-dispatch means of SQ counters (rocprofv3 --pmc, one pass, B = 512 bench steps)')
for (k, cn), (n, s) in sorted(agg.items()):
    print('%-50s %-24s %6d %16.1f' % (k, cn, n, s / n))
PY
cat $O/${TAG}_pmc_lds.txt
