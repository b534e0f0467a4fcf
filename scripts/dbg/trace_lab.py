"""Kernel-trace lab: run each case N times (one sc_gemm dispatch per call); the case order
goes to stdout so rocprofv3's kernel trace can be split per case (scripts/dbg/trace_split.py)."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from sparse_coding__amd.ops import gemm

dev = "cuda"
G, B, n = 8, 2048, 2048
bf = torch.bfloat16
c = torch.empty(G, B, n, device=dev, dtype=bf)
order = []
N = 10
for k in (64, 512):
    x = ((torch.rand(B, k, device=dev) * 2 - 1) * 0.5).to(bf)
    w = ((torch.rand(G, n, k, device=dev) * 2 - 1) * 0.05).to(bf)
    for cfg in (1, 17, 3):
        with gemm.force_shape(cfg):
            for _ in range(N):
                gemm.matmul_nt(x, w, c)
        order.append({"case": f"nt_k{k}_cfg{cfg}", "n": N})
torch.cuda.synchronize()
print(json.dumps(order))
