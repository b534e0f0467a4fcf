"""Per-GPU step time of ensemble-axis sharding at N = 1, 2, 4, 8, measured on ONE GPU.

With ensemble sharding each of N ranks trains G/N models on the all-gathered global batch
of N*B rows (``parallel/ensemble_shard.py``).  The gather of the next batch overlaps the
step, so a rank's step time is the fused step of (G/N models, N*B rows) -- which this
script times directly with the production engine (HIP graph, split-K auto).  Weak-scaling
efficiency at N is t_1 / t_N (the job processes N*B new rows per step).

  python scripts/es_projection.py [--steps 200]
"""

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--models", type=int, default=8)
    ap.add_argument("--d", type=int, default=512)
    ap.add_argument("--ratio", type=int, default=4)
    ap.add_argument("--ns", default="1,2,4,8", help="the N-GPU layouts to measure")
    ap.add_argument("--wsplit", default="auto", help="weight-gradient split-K of the per-rank engine")
    a = ap.parse_args()
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.models.signatures import FunctionalSAE

    dev = "cuda:0"
    torch.manual_seed(0)
    n = a.d * a.ratio
    l1s = np.logspace(-4, -2, a.models)
    models = [FunctionalSAE.init(a.d, n, float(l), device=dev) for l in l1s]
    t1 = None
    for N in [int(v) for v in a.ns.split(",")]:
        if a.models % N:
            continue
        gb = N * a.batch
        ws = a.wsplit if a.wsplit == "auto" else int(a.wsplit)
        eng = FusedSAEEnsemble(models[: a.models // N], FunctionalSAE, lr=1e-3, batch_size=gb, device=dev,
                               wgrad_split=ws)
        eng.enable_graph()
        x = torch.randn(gb, a.d, device=dev).to(torch.bfloat16)
        eng.x_static.copy_(x)
        for _ in range(a.warmup):
            eng.step_static()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            eng.step_static()
        torch.cuda.synchronize()
        ms = 1e3 * (time.perf_counter() - t0) / a.steps
        t1 = t1 or ms
        print(json.dumps({"N": N, "models_per_gpu": a.models // N, "rows_per_step": gb, "wgrad_split": eng.wsplit,
                          "ms_per_step": round(ms, 4), "job_activations_per_s": round(gb / ms * 1e3, 1),
                          "projected_weak_efficiency": round(t1 / ms, 3)}), flush=True)
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
