"""Per-call GEMM routing probe of the TBPTT step: records every plain H.gemm call of one eager
bench step (no mask / bit mask / pending epilogue request -- those must stay on gemm3) at
--rows B, then times each call five ways, interleaved, HIP events, min of three rounds:
  default   the library's own route (hipBLASLt for large plain bf16 problems, else gemm3 /
            gemm2 / skinny),
  gemm3     tile = 5 (the hand-written 256x256 kernels, split-K for fp32 weight gradients),
  blaslt    hipBLASLt with the routing thresholds at 0 (srnn_blaslt_set_min), the library
            heuristic's first algorithm,
  blaslt8   the same, the fastest of the heuristic's first 8 (srnn_blaslt_set_tune(8)),
  skinny    tile = 4 (the small-tile deep-ring NT kernel), for M <= 1024.
Prints one line per call site.  Usage (GPU box, repo root):
  python3 tools/gemm_route_probe.py --rows 64
"""
import argparse
import os
import sys

import torch

os.environ['SRNN_GRAPH'] = '0'          # eager steps: every H.gemm call runs (and is seen)
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, '..'))
sys.path.insert(0, os.path.join(HERE, '..', 'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
import bench  # noqa: E402
import samplernn_hip as H  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--rows', type=int, default=64)
    ap.add_argument('--reps', type=int, default=10)
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    import nn as snn
    import optim
    from trainer import Trainer
    m, pred = bench.make_model(torch.bfloat16)
    pred = pred.to(dev)
    opt = optim.gradient_clipping(torch.optim.Adam(pred.parameters(), lr=1e-3))
    batches = bench.gpu_batches(bench.synth_batches(a.rows, bench.T_SEQ, 64, 2, 0), dev)
    calls = []
    orig = H.gemm
    # an epilogue request (max |C|, column sums, log-softmax) binds the next GEMM to gemm3:
    # such calls are not routing candidates
    pend = [False]
    lib = H.lib()
    ocall = lib.call

    def call(name, *args):
        if name in ('srnn_gemm_amax_next', 'srnn_gemm_amax_blk_next', 'srnn_gemm_csum_next'):
            pend[0] = True
        return ocall(name, *args)
    lib.call = call
    olsm = lib.dll.srnn_gemm_logsoftmax_next

    def lsm_next():
        pend[0] = True
        return olsm()
    lib.dll.srnn_gemm_logsoftmax_next = lsm_next

    def rec(x, y, **kw):
        plain = (kw.get('mask') is None and kw.get('mask_bits') is None and
                 kw.get('bits_out') is None and kw.get('batch', 1) == 1 and not pend[0])
        pend[0] = False
        out = orig(x, y, **kw)
        if plain and len(calls) < 400:
            # the call's own tensors (views included: lda / ldb / ldc refer to their storage;
            # a clone would be compact and the recorded strides would run past it)
            keep = {k: v for k, v in kw.items() if k != 'out'}
            calls.append((x, y, keep, out))
        return out
    H.gemm = rec
    tr = Trainer(pred, snn.sequence_nll_loss_bits, opt, batches[:1], True, None)
    tr.train()
    torch.cuda.synchronize()
    H.gemm = orig
    lib.call = ocall
    lib.dll.srnn_gemm_logsoftmax_next = olsm
    print('rows %d: %d plain gemm calls recorded' % (a.rows, len(calls)), flush=True)
    res = {}
    for rnd in range(3):
        for i, (x, y, kw, out) in enumerate(calls):
            kw2 = dict(kw)
            kw2.pop('tile', None)
            res.setdefault((i, 'default'), []).append(
                timed(lambda: orig(x, y, out=out, **kw2), a.reps))
            try:
                res.setdefault((i, 'gemm3'), []).append(
                    timed(lambda: orig(x, y, out=out, tile=5, **kw2), a.reps))
            except Exception:  # noqa: BLE001 (not eligible)
                pass
            if kw2.get('M', x.shape[1] if kw2.get('transA') else x.shape[0]) <= 1024:
                try:
                    res.setdefault((i, 'skinny'), []).append(
                        timed(lambda: orig(x, y, out=out, tile=4, **kw2), a.reps))
                except Exception:  # noqa: BLE001 (not eligible)
                    pass
            # hipBLASLt for every plain bf16 problem it takes: its heuristic's first
            # algorithm, then the fastest of its first 8 (timed once per shape)
            for tag, tune in (('blaslt', 0), ('blaslt8', 8)):
                lib.dll.srnn_blaslt_set_min(0, 0.0)
                lib.dll.srnn_blaslt_set_tune(tune)
                n0 = lib.dll.srnn_blaslt_calls()
                t = timed(lambda: orig(x, y, out=out, **kw2), a.reps)
                if lib.dll.srnn_blaslt_calls() > n0:
                    res.setdefault((i, tag), []).append(t)
                lib.dll.srnn_blaslt_set_min(4 << 20, 8589934592.0)
                lib.dll.srnn_blaslt_set_tune(0)
    for i, (x, y, kw, out) in enumerate(calls):
        odt = out.dtype
        tA, tB = kw.get('transA', False), kw.get('transB', False)
        M = kw.get('M') or (x.shape[1] if tA else x.shape[0])
        K = kw.get('K') or (x.shape[0] if tA else x.shape[1])
        N = kw.get('N') or (y.shape[0] if tB else y.shape[1])
        line = '%3d M=%6d N=%6d K=%6d tA=%d tB=%d out=%s bias=%d cin=%d' % (
            i, M, N, K, tA, tB, str(odt).replace('torch.', ''), kw.get('bias') is not None,
            kw.get('cin') is not None)
        for v in ('default', 'gemm3', 'skinny', 'blaslt', 'blaslt8'):
            r = res.get((i, v))
            if r:
                line += '  %s %.1f us (%.0f TF/s)' % (v, min(r), 2.0 * M * N * K / min(r) / 1e6)
        print(line, flush=True)


if __name__ == '__main__':
    main()
