"""Lower bound for the 'HIP graph of per-iteration grouped GEMMs + fused FISTA epilogue'
alternative to the persistent Gram solver: time ONLY the
iteration GEMMs y_{t+1} = y_t (D D^T) of config 5 (8 models, B = 2048, n = 1024, 300 iterations)
as one captured graph of grouped MFMA GEMM launches with bf16 output.  Any epilogue
(soft threshold, momentum, gradient offset) can only add to this time."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparse_coding__amd.ops import gemm  # noqa: E402

G, B, n, iters = 8, 2048, 1024, 300
torch.manual_seed(0)
ys = [torch.randn(G, B, n, device="cuda").to(torch.bfloat16) * 0.01 for _ in range(2)]
gram = (torch.randn(G, n, n, device="cuda") * 0.03).to(torch.bfloat16)


def run():
    for i in range(iters):
        gemm.matmul_nn(ys[i % 2], gram, ys[(i + 1) % 2])


run()
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    run()
for _ in range(2):
    g.replay()
torch.cuda.synchronize()
t = time.perf_counter()
reps = 5
for _ in range(reps):
    g.replay()
torch.cuda.synchronize()
ms = 1e3 * (time.perf_counter() - t) / reps
fl = 2.0 * G * B * n * n * iters
print(json.dumps({"what": "graph of 300 grouped GEMMs y <- y (D D^T), config 5 shapes, bf16 out", "ms": round(ms, 2),
                  "tflops": round(fl / ms / 1e9, 1)}))
