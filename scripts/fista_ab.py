"""Gram-form FISTA solve: 32-row vs 16-row workgroups (fista(..., rows=16)), interleaved."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    from sparse_coding__amd.ops import fista as F

    dev = "cuda"
    for n in (512, 1024):
        d = n
        G, B, iters = 8, 2048, 100
        torch.manual_seed(0)
        D = torch.nn.functional.normalize(torch.randn(G, n, d, device=dev), dim=-1)
        X = torch.randn(B, d, device=dev) * 0.3
        lam = torch.full((G,), 1e-3, device=dev)
        eta = F.step_size(D)
        res = {"rt2": [], "rt1": []}
        outs = {}
        for _ in range(5):
            for mode in ("rt2", "rt1"):
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                A, _ = F.fista(X, D, lam, None, iters, eta, backend="hip", with_res=False, form="gram",
                                rows=16 if mode == "rt1" else 0)
                e.record()
                torch.cuda.synchronize()
                res[mode].append(s.elapsed_time(e))
                outs[mode] = A
        diff = (outs["rt2"] - outs["rt1"]).abs().max().item()
        print(json.dumps({"n": n, "d": d, "G": G, "B": B, "iters": iters,
                          **{k: round(statistics.median(v), 3) for k, v in res.items()}, "max_abs_diff": diff}))


if __name__ == "__main__":
    main()
