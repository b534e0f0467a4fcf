"""Per-model code density (mean L0 / n) over the bench's training trajectory."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import bench
from sparse_coding__amd.engine.fused import FusedSAEEnsemble
from sparse_coding__amd.models.signatures import FunctionalSAE

args = bench.parse(["--ring-rows", str(1 << 20)])
dev = torch.device("cuda:0")
torch.manual_seed(0)
n = args.d * args.ratio
models = [FunctionalSAE.init(args.d, n, float(l1), device=dev) for l1 in np.logspace(-4, -2, args.models)]
ring, _ = bench.build_ring(args, dev)
e = FusedSAEEnsemble(models, FunctionalSAE, lr=1e-3, batch_size=args.batch, device=dev)
rec = {}
for s in range(1000):
    out = e.step_batch(ring.sample(args.batch))
    if s in (0, 1, 2, 5, 10, 20, 50, 100, 200, 500, 999):
        rec[s] = [round(float(v), 1) for v in out[:, 4].tolist()]
print(json.dumps({"n": n, "l0_by_step": rec}))
