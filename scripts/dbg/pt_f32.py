import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from sparse_coding__amd.ops import gemm
DEV = "cuda"
torch.manual_seed(0)
for (G, M, N, K) in [(1, 128, 128, 512), (2, 256, 384, 512), (1, 256, 256, 64), (4, 512, 512, 128)]:
    a = torch.randn(G, M, K, device=DEV).to(torch.bfloat16)
    b = torch.randn(G, N, K, device=DEV).to(torch.bfloat16)
    ref = a.float() @ b.float().transpose(1, 2)
    for cfg in (1, 17, 21):
        for dt in (torch.float32, torch.bfloat16):
            out = torch.full((G, M, N), 7.0, device=DEV, dtype=dt)
            with gemm.force_shape(cfg):
                gemm.matmul_nt(a, b, out)
            torch.cuda.synchronize()
            err = float((out.float() - ref).abs().max() / ref.abs().max())
            print(G, M, N, K, "cfg", cfg, dt, "relerr", round(err, 5), "n7", int((out == 7).sum()))
    for mb in (0, 1, 3):
        out = torch.full((G, M, N), 7.0, device=DEV)
        with gemm.force_persistent(True, max_blocks=mb):
            gemm.matmul_nt(a, b, out)
        torch.cuda.synchronize()
        print("  persist mb", mb, "relerr", round(float((out - ref).abs().max() / ref.abs().max()), 5))
