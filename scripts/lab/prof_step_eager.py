"""The headline training step run EAGERLY (no HIP graph) for rocprofv3 counter collection: every
kernel runs in the step's own sequence -- after the kernel that produced its operands, with the
caches as the step leaves them -- unlike scripts/prof_step_kernels.py, which repeats each kernel on
its own."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch

from sparse_coding__amd.engine.fused import FusedSAEEnsemble
from sparse_coding__amd.models.signatures import FunctionalSAE

B, d, n, G = 2048, 512, 2048, 8
dev = "cuda"
torch.manual_seed(0)
models = [FunctionalSAE.init(d, n, float(l1), device=dev) for l1 in np.logspace(-4, -2, G)]
e = FusedSAEEnsemble(models, FunctionalSAE, batch_size=B, device=dev, track_feature_counts=False)
feats = torch.nn.functional.normalize(torch.randn(4096, d, device=dev), dim=-1)
xs = [((torch.relu(torch.randn(B, 4096, device=dev) - 2.0) * 3.0) @ feats).to(torch.bfloat16) for _ in range(4)]
for i in range(24):
    e.step_batch(xs[i % 4])
torch.cuda.synchronize()
print("done")
