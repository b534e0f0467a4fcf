"""Fixed cost of the fused step tail: one step_tail launch (2 sets, d = 512, G = 8) timed in isolation
for n = 128 .. 2048 rows per model, with and without the next-batch gather; the intercept of time vs
bytes is the per-launch fixed part (launch, loss / bias blocks, tickets, gather latency)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from sparse_coding__amd.ops import adam as adam_ops


def _padded(shape, dtype, k, stagger):
    """A tensor placed k x `stagger` bytes into a slightly larger allocation (staggers the start of each
    stream the kernel walks in lockstep)."""
    numel = 1
    for x in shape:
        numel *= x
    es = torch.tensor([], dtype=dtype).element_size()
    off = (k * stagger) // es
    buf = torch.empty(numel + off, device="cuda", dtype=dtype)
    return buf[off:off + numel].view(*shape)


def run(n, gather, G=8, d=512, B=2048, iters=200, norms_=(False, True), gbf=False, stagger=0, parts=1):
    dev = "cuda"
    f = dict(device=dev, dtype=torch.float32)
    sets = []
    for norm in norms_:
        mk = lambda k, dt=torch.float32: _padded((G, n, d), dt, k, stagger)
        p_, g_, m_, v_, sh_ = mk(0), mk(1, torch.bfloat16 if gbf else torch.float32), mk(2), mk(3), mk(4, torch.bfloat16)
        p_.normal_()
        g_.copy_(torch.randn(G, n, d, **f) * 1e-3)
        m_.zero_()
        v_.zero_()
        sets.append(dict(p=p_, g=g_, m=m_, v=v_, shadow=sh_, norms=None, norm=norm))
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
    tickets = [torch.zeros(adam_ops.TICKET_INTS, device=dev, dtype=torch.int32) for _ in range(parts)]
    bsq_parts = [torch.zeros(2, G // parts, n // 32, **f) for _ in range(parts)]
    gat = None
    if gather:
        ring = torch.randn(1 << 18, d, device=dev).to(torch.bfloat16)
        perm = torch.randperm(1 << 18, device=dev)
        ep0 = torch.zeros(1, device=dev, dtype=torch.int32)
        gout = torch.empty(B, d, device=dev, dtype=torch.bfloat16)
        gat = (ring, perm, ep0, gout)

    def call():
        if parts == 1:
            adam_ops.step_tail(sets, lr, 0.9, 0.999, 1e-8, step, bias, bm, bv, colpart, enc_part, dec_part, l1, bdec,
                               out, B, 1.0 / B, bsq, ticket, gather=gat)
            return
        h = G // parts  # (lab) the same update as `parts` launches over model slices
        for q in range(parts):
            sl = slice(q * h, (q + 1) * h)
            ss = [{k: (v[sl] if torch.is_tensor(v) and v.dim() == 3 else v) for k, v in st.items()} for st in sets]
            adam_ops.step_tail(ss, lr[sl], 0.9, 0.999, 1e-8, step, bias[sl], bm[sl], bv[sl], colpart[sl],
                               enc_part[sl], dec_part[sl], l1[sl], bdec[sl], out[sl], B, 1.0 / B,
                               bsq[:, sl].contiguous() if False else bsq_parts[q], tickets[q])

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
    mb = len(norms_) * G * n * d * (28 if gbf else 30) / 1e6
    return {"n": n, "d": d, "sets": len(norms_), "gbf16": gbf, "gather": gather, "stagger": stagger, "parts": parts,
            "us": round(us, 2),
            "MB": round(mb, 1), "TBps": round(mb / us, 2)}


if "--topk" in sys.argv:  # the top-k tail's shape: one normalised set, d = 768, n = 6144, bf16 gradient
    for parts in (1, 2, 4):
        print(json.dumps(run(6144, False, d=768, norms_=(True,), gbf=True, parts=parts)), flush=True)
    print(json.dumps(run(3072, False, d=768, norms_=(True,), gbf=True)), flush=True)
    sys.exit(0)
for gather in (False, True):
    for n in (128, 256, 512, 1024, 2048):
        print(json.dumps(run(n, gather)), flush=True)
