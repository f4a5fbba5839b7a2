"""Timing experiments on the XCD GRU sweeps (SRNN_GX_EXP variants; results are invalid under
any nonzero value): us per step of the forward and backward sweep at B rows, D = 1024, 64
frames.  Usage: python tools/gx_exp.py B1,B2 exp1,exp2,..."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

Bs = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else '128').split(',')]
exps = (sys.argv[2] if len(sys.argv) > 2 else '0').split(',')
for B in Bs:
    for e in exps:
        os.environ['SRNN_GX_EXP'] = e
        r = bench.gru_sweep_roofline('cuda', B=B)
        print('B=%d exp=%s fwd %.2f us/step bwd %.2f us/step' % (
            B, e, r['fwd']['us_per_step'], r['bwd']['us_per_step']), flush=True)
os.environ['SRNN_GX_EXP'] = '0'
