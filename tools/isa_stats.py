"""Per-kernel ISA statistics from a hipcc -save-temps .s file: VGPRs, scratch, MFMA count,
s_waitcnt vmcnt immediates, barriers.   python3 tools/isa_stats.py file.s [name-substring]"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ''
for m in re.finditer(r'^(_Z\S+):\s+;\s+@', s, re.M):
    name = m.group(1)
    if pat not in name:
        continue
    start = m.end()
    end = s.find('.Lfunc_end', start)
    body = s[start:end]
    tail = s[end:end + 6000]
    vg = re.search(r'; NumVgprs:\s+(\d+)', tail)
    ag = re.search(r'; NumAgprs:\s+(\d+)', tail)
    sp = re.search(r'; ScratchSize:\s+(\d+)', tail)
    print(name[:90])
    print('   vgpr %s agpr %s scratch %s  mfma %d  s_barrier %d  ds_read %d  glds %d  lines %d' % (
        vg and vg.group(1), ag and ag.group(1), sp and sp.group(1), len(re.findall(r'v_mfma', body)),
        len(re.findall(r's_barrier', body)), len(re.findall(r'ds_read', body)),
        len(re.findall(r'global_load_lds', body)), body.count('\n')))
    print('   vmcnt:', Counter(re.findall(r'vmcnt\((\d+)\)', body)).most_common(14))
    print('   lgkmcnt:', Counter(re.findall(r'lgkmcnt\((\d+)\)', body)).most_common(8))
