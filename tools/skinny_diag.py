import os, sys, torch
sys.path.insert(0, 'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd')
import samplernn_hip as H
T = torch.bfloat16
for (M, N, K) in [(128, 4096, 1024), (128, 16384, 1024)]:
    a = torch.randn(M, K, device='cuda').to(T); w = torch.randn(N, K, device='cuda').to(T)
    b = torch.randn(N, device='cuda'); out = torch.empty(M, N, device='cuda')
    for _ in range(20):
        H.linear(a, w, bias=b, out=out)
    torch.cuda.synchronize()
    print(M, N, K, flush=True)
    H.lib().dll.srnn_skinny_diag_dump()
