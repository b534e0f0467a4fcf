"""Row-Adam bandwidth at equal bytes for d = 512 / 768 / 1024 (norm rows, bf16 or fp32 gradient)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparse_coding__amd.ops import adam as adam_ops  # noqa: E402


def run(G, n, d, gdt):
    p = torch.randn(G, n, d, device="cuda")
    g = torch.randn(G, n, d, device="cuda").to(gdt)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    sh = torch.empty(G, n, d, device="cuda", dtype=torch.bfloat16)
    nr = torch.empty(G, n, device="cuda")
    lr = torch.full((G,), 1e-3, device="cuda")
    st = [dict(p=p, g=g, m=m, v=v, shadow=sh, norms=nr, norm=True)]
    for _ in range(3):
        adam_ops.adam_rows(st, lr, 3)
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(20):
        adam_ops.adam_rows(st, lr, 3)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 20
    nbytes = G * n * d * (4 * 6 + 2 + g.element_size())
    return {"G": G, "n": n, "d": d, "grad": str(gdt), "us": round(us, 1), "TBps": round(nbytes / us / 1e6, 2)}


for gdt in (torch.float32, torch.bfloat16):
    for (n, d) in ((9216, 512), (6144, 768), (4608, 1024)):
        print(json.dumps(run(8, n, d, gdt)))
