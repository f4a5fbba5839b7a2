"""Timing decomposition of the da1 GEMM at the B = 512 TBPTT shape (M = 512 x 1024 rows,
N = K = 1024, bf16, NT: da2 . W_hid^T with W_hid^T stored k-contiguous): the step's form (bf16
ReLU mask read from a1 + max |C|) against the same GEMM with parts of its epilogue removed,
interleaved in one process, HIP events on the launching stream.  The step's default since
round 5: a1's mask as grouped bits, staged by LDS-DMA (SRNN_A1_BITS).

    python tools/da1_probe.py [reps]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))
import samplernn_hip as H  # noqa: E402


def main(reps=10):
    dev = torch.device('cuda:0')
    g = torch.Generator(device=dev).manual_seed(5)
    M, N, K = 512 * 1024, 1024, 1024
    bf = torch.bfloat16
    da2 = (torch.randn(M, K, device=dev, generator=g) * 0.01).to(bf)
    Wt = (torch.randn(N, K, device=dev, generator=g) * 0.03).to(bf)       # W_hid^T, k-contiguous
    a1 = torch.relu(torch.randn(M, N, device=dev, generator=g)).to(bf)
    bits = H.relu_bits(M, N, dev)
    H.lib().call('srnn_relu_bits', H.BF16, H.ptr(a1), N, M, N, H.ptr(bits), bits.stride(0),
                 H.stream())
    gbits = H.relu_bits_grouped(M, N, dev)                 # the step's default (SRNN_A1_BITS)
    H.lib().call('srnn_relu_bits', H.BF16, H.ptr(a1), N, M, N, H.ptr(gbits), 0, H.stream())
    amax = torch.zeros(1, device=dev, dtype=torch.int32)
    s = torch.cuda.current_stream()

    def form(name, env, mask=None, mbits=None, want_amax=False):
        return name, env, mask, mbits, want_amax

    forms = [
        form('grouped bits (LDS-DMA) + max|C| (step default)', {}, mbits=gbits, want_amax=True),
        form('grouped bits, no max', {}, mbits=gbits),
        form('bf16 mask + max|C| (SRNN_A1_BITS=0)', {}, mask=a1, want_amax=True),
        form('  + fragment prefetch (SRNN_G3_AMX_PF=1)', {'SRNN_G3_AMX_PF': '1'}, mask=a1,
             want_amax=True),
        form('bf16 mask, no max', {}, mask=a1),
        form('row-major bits, no max', {}, mbits=bits),
        form('no mask, no max, gemm3 (SRNN_BLASLT=0)', {'SRNN_BLASLT': '0'}),
        form('no mask, no max, hipBLASLt', {}),
        form('grouped bits + max, no epilogue (SRNN_G3DIAG=8)', {'SRNN_G3DIAG': '8'},
             mbits=gbits, want_amax=True),
    ]
    res = {f[0]: [] for f in forms}
    for rnd in range(3):
        for name, env, mask, mbits, want_amax in forms:
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            try:
                ts = []
                for r in range(reps + 1):
                    if want_amax:
                        amax.zero_()
                        H.lib().call('srnn_gemm_amax_next', H.ptr(amax))
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    if mbits is not None:
                        H.gemm(da2, Wt, transB=True, mask_bits=mbits, out_dtype=bf)
                    else:
                        H.gemm(da2, Wt, transB=True, mask=mask, out_dtype=bf)
                    e1.record(s)
                    if want_amax:
                        H.lib().dll.srnn_gemm_amax_taken()
                    e1.synchronize()
                    if r:
                        ts.append(e0.elapsed_time(e1))
                res[name].append(sorted(ts)[len(ts) // 2])
            finally:
                for k, v in old.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
    flop = 2.0 * M * N * K
    print('# da1 GEMM forms, M=%d N=%d K=%d bf16 NT, median ms of %d launches per round, 3 rounds'
          % (M, N, K, reps))
    for name, _, _, _, _ in forms:
        v = res[name]
        print('%-48s %s  -> %.1f TFLOP/s (best)' % (name, ' '.join('%.4f' % x for x in v),
                                                  flop / min(v) / 1e9))


if __name__ == '__main__':
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 10)
