"""LISTA (or, with --residual, residual-denoising) ensemble step: UnrolledEnsemble (grouped MFMA
GEMMs) vs the vmap(grad) FunctionalEnsemble on the same GPU (8 models, d=512, n=2048, 3 layers, B=2048)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sparse_coding__amd.engine.ensemble import FunctionalEnsemble
from sparse_coding__amd.engine.optim import adam
from sparse_coding__amd.engine.unrolled import UnrolledEnsemble
from sparse_coding__amd.models.lista import FunctionalLISTADenoisingSAE, FunctionalResidualDenoisingSAE

S = FunctionalResidualDenoisingSAE if "--residual" in sys.argv else FunctionalLISTADenoisingSAE


def timeit(fn, steps=30, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t) / steps


torch.manual_seed(0)
d, n, B, G, L = 512, 2048, 2048, 8, 3
models = [S.init(d, n, L, float(l1), device="cuda") for l1 in torch.logspace(-4, -2, G)]
x = torch.randn(B, d, device="cuda")
eng = UnrolledEnsemble(models, S, device="cuda")
ms = timeit(lambda: eng.step_batch(x))


def autograd_step():  # the engine's torch-autograd path over the same kernels (before round 6's explicit step)
    g, _ = eng.grads(x)
    eng.apply_grads(g)


if "--only-unrolled" in sys.argv:
    print(json.dumps({"model": S.__name__, "unrolled_ms_per_step": round(ms, 3)}))
    sys.exit(0)
ms_a = timeit(autograd_step)
ens = FunctionalEnsemble(models, S, adam, {"lr": 1e-3}, device="cuda")
ms_e = timeit(lambda: ens.step_batch(x))
print(json.dumps({"config": f"{'residual-denoising' if S is FunctionalResidualDenoisingSAE else 'LISTA'} {G} models d={d} n={n} layers={L} B={B}", "unrolled_ms_per_step": round(ms, 3), "autograd_path_ms_per_step": round(ms_a, 3),
                  "eager_vmap_ms_per_step": round(ms_e, 3), "speedup": round(ms_e / ms, 2),
                  "unrolled_act_per_s": round(B / ms * 1e3)}))
