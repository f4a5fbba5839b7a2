"""Compressed instruction flow of one kernel in a hipcc -save-temps .s file: runs of MFMA /
ds_read / global_load_lds / VALU collapsed, waits, barriers, branches and labels kept.
  python3 tools/isa_flow.py file.s exact_symbol [max_lines]"""
import re
import sys

s = open(sys.argv[1]).read()
name = sys.argv[2]
lim = int(sys.argv[3]) if len(sys.argv) > 3 else 400
i = s.index('\n' + name + ':')
body = s[i:s.find('.Lfunc_end', i)].split('\n')
out, run, cnt = [], None, 0


def flush():
    global run, cnt
    if run:
        out.append('   %-14s x%d' % (run, cnt))
    run, cnt = None, 0


for ln in body:
    t = ln.strip()
    if not t or t.startswith(';') or t.startswith('.'):
        if t.startswith('.LBB'):
            flush()
            out.append(t.split(';')[0])
        continue
    op = t.split()[0]
    key = None
    if op.startswith('v_mfma'):
        key = 'mfma'
    elif op.startswith('ds_read') or op.startswith('ds_load'):
        key = 'ds_read'
    elif op.startswith('global_load_lds'):
        key = 'glds'
    elif op.startswith('global_store') or op.startswith('buffer_store'):
        key = 'store'
    elif op.startswith('global_load') or op.startswith('buffer_load'):
        key = 'vload'
    elif op.startswith('scratch'):
        key = 'SCRATCH'
    elif op.startswith('v_') or op.startswith('s_') and op not in (
            's_waitcnt', 's_barrier', 's_cbranch_scc0', 's_cbranch_scc1', 's_branch',
            's_cbranch_vccz', 's_cbranch_vccnz', 's_cbranch_execz', 's_setprio', 's_endpgm'):
        key = 'alu'
    if key:
        if key != run:
            flush()
            run = key
        cnt += 1
        continue
    flush()
    out.append('   ' + t.split(';')[0])
flush()
print('\n'.join(out[:lim]))
