"""Launch only the bench's dominant kernel (same shape/dtype/epilogue as bench.py's roofline
leg) so that rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) see it in isolation.

  rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run -- python tools/archive/roofline_kernel.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    which = sys.argv[1] if len(sys.argv) > 1 else 'gemm'
    if which == 'gemm':
        ms = bench.kernel_roofline_gemm(dev, 128 * 1024, 1024, 1024, torch.bfloat16, reps=5)
        print('gemm %.3f ms/launch' % ms)
    else:
        raise SystemExit('unknown kernel ' + which)


if __name__ == '__main__':
    main()
