"""One generation run for rocprofv3 traces / PMC passes: configs[2] (3-tier, FS [16, 4],
cond 43) or, with 'e', configs[4] (4-tier, FS [16, 4, 4], look-ahead cond 86); 128
utterances, dim 1024:  python tools/gen_prof.py fp32|bf16 [n_cond] [e]."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
import torch  # noqa: E402
import bench  # noqa: E402

dt = torch.float32 if sys.argv[1] == 'fp32' else torch.bfloat16
n_cond = int(sys.argv[2]) if len(sys.argv) > 2 else 750
cfg_e = len(sys.argv) > 3 and sys.argv[3] == 'e'
fs, cd = ((16, 4, 4), 86) if cfg_e else ((16, 4), 43)
t, _ = bench.run_gen(torch.device('cuda', 0), 128, n_cond, dt, fs, cd)
print('gen %s%s: %.3f s for %d samples/row' % (sys.argv[1], ' config e' if cfg_e else '', t,
                                              n_cond * int(torch.tensor(fs).prod())))
