"""GEMM lab: where does a step GEMM spend its time?  Interleaved timing (one process,
several rounds, median) of the grouped GEMM kernels over K, so the fixed per-tile cost
(prologue + epilogue) separates from the per-K-step main-loop cost.

python scripts/gemm_lab.py [--rounds 5] [--out gpurun_out/gemm_lab.jsonl] [--which enc,dec,...]
"""

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--G", type=int, default=8)
    ap.add_argument("--B", type=int, default=2048)
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--d", type=int, default=512)
    ap.add_argument("--out", default="gpurun_out/gemm_lab.jsonl")
    ap.add_argument("--which", default="")
    ap.add_argument("--cfgs", default="")
    a = ap.parse_args()
    from sparse_coding__amd.ops import gemm

    torch.manual_seed(0)
    dev = "cuda"
    G, B, n, d = a.G, a.B, a.n, a.d
    bf = torch.bfloat16
    cases = {}
    # encoder-shaped (M = B, N = n, K = k): plain bf16 out vs fused ENC epilogue, over K
    for k in (64, 128, 256, 512):
        x = (torch.rand(B, k, device=dev) * 2 - 1).to(bf)
        w = (torch.rand(G, n, k, device=dev) * 2 - 1).to(bf)
        c = torch.empty(G, B, n, device=dev, dtype=bf)
        bias = torch.zeros(G, n, device=dev) - 0.1
        part = torch.empty(G, (B // 128) * (n // 128), 2, device=dev)
        mask = torch.empty(gemm.code_mask_shape(G, B, n), device=dev, dtype=torch.int64)
        fl = 2.0 * G * B * n * k
        cases[f"nt_bf16_k{k}"] = (lambda x=x, w=w, c=c: gemm.matmul_nt(x, w, c), fl)
        cases[f"enc_k{k}"] = (lambda x=x, w=w, c=c, bias=bias, part=part, mask=mask:
                              gemm.encode_relu(x, w, bias, c, part, None, None, mask_out=mask), fl)
        cases[f"torch_k{k}"] = (lambda x=x, w=w, c=c: torch.matmul(x, w.transpose(1, 2), out=c), fl)
    # decoder-shaped (M = B, N = d, K = n)
    for k in (512, 1024, 2048):
        cc = (torch.rand(G, B, k, device=dev) * 2 - 1).to(bf)
        wh = (torch.rand(G, k, d, device=dev) * 2 - 1).to(bf)
        x = (torch.rand(B, d, device=dev) * 2 - 1).to(bf)
        r = torch.empty(G, B, d, device=dev, dtype=bf)
        part = torch.empty(G, (B // 128) * (d // 128), device=dev)
        fl = 2.0 * G * B * k * d
        cases[f"dec_k{k}"] = (lambda cc=cc, wh=wh, x=x, r=r, part=part: gemm.decode_residual(cc, wh, x, r, part), fl)
        cases[f"nn_bf16_k{k}"] = (lambda cc=cc, wh=wh, r=r: gemm.matmul_nn(cc, wh, r), fl)
        cases[f"torch_dec_k{k}"] = (lambda cc=cc, wh=wh, r=r: torch.matmul(cc, wh, out=r), fl)
    # weight-gradient-shaped (M = n, N = d, K = B)
    for kb in (512, 1024, 2048):
        cc = (torch.rand(G, kb, n, device=dev) * 2 - 1).to(bf)
        rr = (torch.rand(G, kb, d, device=dev) * 2 - 1).to(bf)
        g1 = torch.empty(G, n, d, device=dev)
        g2 = torch.empty(G, n, d, device=dev)
        fl = 2 * 2.0 * G * kb * n * d
        cases[f"wgrad2_k{kb}"] = (lambda cc=cc, rr=rr, g1=g1, g2=g2:
                                  gemm.weight_grads([[(cc, rr)], [(cc, rr)]], [g1, g2], 1.0), fl)
    # the step GEMMs at the headline shape through the tile kernel vs the persistent kernel
    x = (torch.rand(B, d, device=dev) * 2 - 1).to(bf)
    we = ((torch.rand(G, n, d, device=dev) * 2 - 1) * 0.05).to(bf)
    wd = torch.nn.functional.normalize(torch.randn(G, n, d, device=dev), dim=-1).to(bf)
    bias = torch.zeros(G, n, device=dev) - 0.02
    c = torch.empty(G, B, n, device=dev, dtype=bf)
    part = torch.empty(G, (B // 128) * (n // 128), 2, device=dev)
    cnt = torch.empty(G, B // 128, n, device=dev)
    cmask = torch.empty(gemm.code_mask_shape(G, B, n), device=dev, dtype=torch.int64)
    r = torch.empty(G, B, d, device=dev, dtype=bf)
    dpart = torch.empty(G, (B // 128) * (d // 128), device=dev)
    dpre = torch.empty(G, B, n, device=dev, dtype=bf)
    colpart = torch.empty(G, B // 128, n, device=dev)
    l1 = torch.full((G,), 1e-3, device=dev)
    gd = torch.empty(G, n, d, device=dev)
    ge = torch.empty(G, n, d, device=dev)
    fl = 2.0 * G * B * n * d
    step_ops = {
        "enc": (lambda: gemm.encode_relu(x, we, bias, c, part, None, None, mask_out=cmask), fl),
        "enc_cnt": (lambda: gemm.encode_relu(x, we, bias, c, part, cnt, None, mask_out=cmask), fl),
        "dec": (lambda: gemm.decode_residual(c, wd, x, r, dpart), fl),
        "dc": (lambda: gemm.code_grad(r, wd, c, l1, dpre, colpart, mask=cmask), fl),
        "wgrad": (lambda: gemm.weight_grads([[(c, r)], [(dpre, x)]], [gd, ge], 1e-6), 2 * fl),
        "ntbf16": (lambda: gemm.matmul_nt(x, we, c), fl),
    }
    gemm.encode_relu(x, we, bias, c, part, None, None, mask_out=cmask)
    modes = [("tile", lambda: gemm.force_shape(1))]
    if a.cfgs:  # explicit tile-kernel configurations (block shape | pipeline << 2) instead
        modes = [(f"cfg{c}", lambda c=int(c): gemm.force_shape(c)) for c in a.cfgs.split(",")]
    cases["step_torch_enc"] = (lambda: torch.matmul(x, we.transpose(1, 2), out=c), fl)
    cases["step_torch_dec"] = (lambda: torch.matmul(c, wd, out=r), fl)
    cases["step_torch_wgrad"] = (lambda: (torch.matmul(c.transpose(1, 2), r),
                                          torch.matmul(dpre.transpose(1, 2), x)), 2 * fl)
    for name, (fn, f) in step_ops.items():
        for mode, ctx in modes:
            def run(fn=fn, ctx=ctx):
                with ctx():
                    fn()
            cases[f"step_{name}_{mode}"] = (run, f)
    names = [k for k in cases if not a.which or any(k.startswith(w) for w in a.which.split(","))]
    res = {k: [] for k in names}
    for _ in range(a.rounds):
        for k in list(names):
            try:
                res[k].append(timeit(cases[k][0]))
            except Exception as e:  # a configuration the library does not instantiate
                print(json.dumps({"case": k, "error": str(e)[:120]}), flush=True)
                names.remove(k)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        for k in names:
            med = statistics.median(res[k])
            rec = {"case": k, "median_us": round(med, 2), "min_us": round(min(res[k]), 2),
                   "tflops": round(cases[k][1] / med / 1e6, 1)}
            print(json.dumps(rec), flush=True)
            f.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
