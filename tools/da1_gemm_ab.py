"""The MLP's da1 GEMM (da1 = (da2 . W_hid) * [a1 > 0], bf16 out, M = B*1024, N = K = 1024) in
its variants, interleaved in one process: ReLU mask from the bf16 activations or none, with or
without the max |C| epilogue (srnn_gemm_amax_next), with or without the unit-1 prefetch
(SRNN_G3_AMX_PF / SRNN_G3_PF).  HIP events around 5 back-to-back launches."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..',
                                'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
import samplernn_hip as H  # noqa: E402


def bench(fn, reps=5):
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
    D = 1024
    for B in (512, 128):
        M = B * 1024
        da2 = ((torch.rand(M, D, device='cuda') * 2 - 1) * 1e-3).bfloat16()
        W = ((torch.rand(D, D, device='cuda') * 2 - 1) * 0.03).bfloat16()
        a1 = (torch.rand(M, D, device='cuda') * 2 - 1).bfloat16()
        amax = torch.zeros(1, device='cuda', dtype=torch.int32)

        Wt = W.t().contiguous()

        def run(mask, amx, nt=False):
            if amx:
                H.lib().call('srnn_gemm_amax_next', H.ptr(amax))
            if nt:      # the same product with W_hid^T stored k-contiguous (NT shape)
                H.gemm(da2, Wt, transB=True, mask=a1 if mask else None, out_dtype=torch.bfloat16)
            else:
                H.gemm(da2, W, mask=a1 if mask else None, out_dtype=torch.bfloat16)
            if amx:
                assert H.lib().dll.srnn_gemm_amax_taken()
        variants = [('mask', True, False, False, {}),
                    ('mask+amax', True, True, False, {'SRNN_G3_AMX_PF': '0'}),
                    ('mask+amax+pf', True, True, False, {'SRNN_G3_AMX_PF': '1'}),
                    ('no mask', False, False, False, {}),
                    ('NT mask', True, False, True, {}),
                    ('NT mask+amax', True, True, True, {'SRNN_G3_AMX_PF': '0'}),
                    ('NT mask+amax+pf', True, True, True, {'SRNN_G3_AMX_PF': '1'}),
                    ('NT no mask', False, False, True, {})]
        ref = None
        res = {}
        for _ in range(3):
            for name, mk, amx, nt, env in variants:
                old = {k: os.environ.get(k) for k in env}
                os.environ.update(env)
                res.setdefault(name, []).append(bench(lambda: run(mk, amx, nt)))
                for k, v in old.items():
                    if v is None:
                        os.environ.pop(k)
                    else:
                        os.environ[k] = v
        for name, *_ in variants:
            r = res[name]
            print('B=%d %-14s %s us (min %.1f)' % (B, name, ['%.1f' % x for x in r], min(r)),
                  flush=True)


if __name__ == '__main__':
    main()
