"""Config 5 (FISTA dictionary learning, d = n = 1024, 8 models, B = 2048, 300 iterations): the whole
training step with the GPU dictionary-update hot path (``ops.fista.gram_solve``) against the previous
path (``fista()`` + fp32 residual + fp32 D^T D eta + fp32 operand copies), alternating on one box, plus
the solve alone.  One JSON line: step ms per variant, solve ms, step - solve.

    python scripts/fista_step_ab.py [--rounds 3 --steps 20]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--iters", type=int, default=300)
    a = ap.parse_args()
    from sparse_coding__amd.data.ring import DeviceRing
    from sparse_coding__amd.engine.trainer import EnsembleTrainer
    from sparse_coding__amd.models.fista import FunctionalFista
    from sparse_coding__amd.ops import fista as F

    dev = "cuda:0"
    torch.manual_seed(0)
    d = n = 1024
    B, G = 2048, 8
    l1s = np.logspace(-4, -2, G)
    ring = DeviceRing(1 << 19, d, device=dev, seed=5)
    ring.fill(lambda: torch.randn(65536, d, device=dev) * 0.1)
    xbuf = torch.empty(B, d, device=dev, dtype=torch.bfloat16)
    hot_ok = F.gram_solve_ok
    trainers = {}
    for name in ("hot", "old"):
        models = [FunctionalFista.init(d, n, float(l1), device=dev) for l1 in l1s]
        trainers[name] = EnsembleTrainer(models, FunctionalFista, batch_size=B, device=dev, fista_iters=a.iters,
                                         fista_backend="hip")

    def run(name, steps):
        F.gram_solve_ok = hot_ok if name == "hot" else (lambda *args: False)
        tr = trainers[name]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            tr.step(ring.sample(B, out=xbuf))
        torch.cuda.synchronize()
        return 1e3 * (time.perf_counter() - t0) / steps

    for name in trainers:
        run(name, a.warmup)
    ms = {name: [] for name in trainers}
    for _ in range(a.rounds):
        for name in trainers:
            ms[name].append(run(name, a.steps))
    F.gram_solve_ok = hot_ok
    D = torch.nn.functional.normalize(torch.randn(G, n, d, device=dev), dim=-1)
    x = ring.sample(B).float()
    eta = F.step_size(D)
    lam = torch.tensor(l1s, device=dev, dtype=torch.float32)
    F.fista(x, D, lam, None, a.iters, eta, backend="hip", with_res=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        F.fista(x, D, lam, None, a.iters, eta, backend="hip", with_res=False)
    torch.cuda.synchronize()
    solve = 1e3 * (time.perf_counter() - t0) / 3
    med = {k: statistics.median(v) for k, v in ms.items()}
    print(json.dumps({"config": "5: FISTA dictionary learning d=n=1024, 8 models, B=2048, 300 iterations",
                      "ms_per_step": {k: round(v, 3) for k, v in med.items()},
                      "runs": {k: [round(x, 3) for x in v] for k, v in ms.items()},
                      "solve_ms": round(solve, 3),
                      "step_minus_solve_ms": {k: round(v - solve, 3) for k, v in med.items()},
                      "activations_per_s": {k: round(B / (v / 1e3), 1) for k, v in med.items()}}), flush=True)


if __name__ == "__main__":
    main()
