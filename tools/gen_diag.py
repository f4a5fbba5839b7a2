"""Phase stamps of one steady-state persistent generation launch (SRNN_GEN_DIAG=n, timing
diagnostics only): python tools/gen_diag.py bf16|fp32 [launch_index]"""
import os
import sys
os.environ['SRNN_GEN_DIAG'] = sys.argv[2] if len(sys.argv) > 2 else '30'
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
import torch  # noqa: E402
import bench  # noqa: E402
import samplernn_hip as H  # noqa: E402

dt = torch.float32 if sys.argv[1] == 'fp32' else torch.bfloat16
bench.run_gen(torch.device('cuda', 0), 128, 20, dt)
torch.cuda.synchronize()
H.lib().dll.srnn_gen_diag_dump()
