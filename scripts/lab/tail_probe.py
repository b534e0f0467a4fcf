"""Fixed cost of the fused step tail: one step_tail launch (2 sets, d = 512, G = 8) timed in isolation
for n = 128 .. 2048 rows per model, with and without the next-batch gather; the intercept of time vs
bytes is the per-launch fixed part (launch, loss / bias blocks, tickets, gather latency)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from sparse_coding__amd.ops import adam as adam_ops


def run(n, gather, G=8, d=512, B=2048, iters=200):
    dev = "cuda"
    f = dict(device=dev, dtype=torch.float32)
    sets = []
    for norm in (False, True):
        sets.append(dict(p=torch.randn(G, n, d, **f), g=torch.randn(G, n, d, **f) * 1e-3, m=torch.zeros(G, n, d, **f),
                         v=torch.zeros(G, n, d, **f), shadow=torch.empty(G, n, d, device=dev, dtype=torch.bfloat16),
                         norms=None, norm=norm))
    lr = torch.full((G,), 1e-3, **f)
    step = torch.zeros(1, device=dev, dtype=torch.int32)
    bias, bm, bv = torch.zeros(G, n, **f), torch.zeros(G, n, **f), torch.zeros(G, n, **f)
    tm = B // 128
    colpart = torch.randn(G, tm, n, **f)
    enc_part = torch.rand(G, tm * (n // 128), 2, **f)
    dec_part = torch.rand(G, tm * (d // 128), **f)
    l1 = torch.full((G,), 1e-3, **f)
    bdec = torch.zeros(G, **f)
    out = torch.zeros(G, 6, **f)
    bsq = torch.zeros(2, G, n // 32, **f)
    ticket = torch.zeros(adam_ops.TICKET_INTS, device=dev, dtype=torch.int32)
    gat = None
    if gather:
        ring = torch.randn(1 << 18, d, device=dev).to(torch.bfloat16)
        perm = torch.randperm(1 << 18, device=dev)
        ep0 = torch.zeros(1, device=dev, dtype=torch.int32)
        gout = torch.empty(B, d, device=dev, dtype=torch.bfloat16)
        gat = (ring, perm, ep0, gout)

    def call():
        adam_ops.step_tail(sets, lr, 0.9, 0.999, 1e-8, step, bias, bm, bv, colpart, enc_part, dec_part, l1, bdec,
                           out, B, 1.0 / B, bsq, ticket, gather=gat)

    for _ in range(3):
        call()
    torch.cuda.synchronize()
    per = 20  # launches per graph: the host's Python launch cost stays out of the timing
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(per):
            call()
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters // per):
        gr.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (per * (iters // per))
    mb = 2 * G * n * d * 30 / 1e6
    return {"n": n, "gather": gather, "us": round(us, 2), "MB": round(mb, 1), "TBps": round(mb / us, 2)}


for gather in (False, True):
    for n in (128, 256, 512, 1024, 2048):
        print(json.dumps(run(n, gather)), flush=True)
