"""Phase timestamps of one persistent generation launch (SRNN_GEN_DIAG=n arms the n-th
launch of the process; workgroup 0's stamps, then per-workgroup start / group-known /
prologue-done spreads), printed by srnn_gen_diag_dump:
    SRNN_GEN_DIAG=20 python tools/gen_diag.py [bf16|fp32]"""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
import torch  # noqa: E402
import bench  # noqa: E402
import samplernn_hip as H  # noqa: E402

dt = torch.float32 if len(sys.argv) > 1 and sys.argv[1] == 'fp32' else torch.bfloat16
bench.run_gen(torch.device('cuda', 0), 128, 8, dt)
torch.cuda.synchronize()
H.lib().dll.srnn_gen_diag_dump()
