"""Why do the step GEMMs run slower inside the training step than in isolation?  Phase A runs
engine steps; phase B repeats each step GEMM alone on the engine's REAL buffers; phase C the
same on random-code buffers.  Per-kernel durations come from the rocprofv3 kernel trace
(phases separated by markers: a tiny torch kernel count)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch

from sparse_coding__amd.engine.fused import FusedSAEEnsemble
from sparse_coding__amd.models.signatures import FunctionalSAE
from sparse_coding__amd.ops import gemm

import bench

B, d, n, G = 2048, 512, 2048, 8
dev = "cuda"
torch.manual_seed(0)
models = [FunctionalSAE.init(d, n, float(l), device=dev) for l in np.logspace(-4, -2, G)]
e = FusedSAEEnsemble(models, FunctionalSAE, batch_size=B, device=dev)
args = bench.parse([])
ring, _ = bench.build_ring(args, dev)
xs = [ring.sample(B).to(torch.bfloat16).contiguous() for _ in range(4)]
for i in range(200):  # train a little so the codes are sparse like the bench's
    e.step_batch(xs[i % 4])
torch.cuda.synchronize()
x = xs[0]
for i in range(30):   # phase A
    e.step_batch(xs[i % 4])
torch.cuda.synchronize()
torch.zeros(1, device=dev).add_(1)
e.forward(x)
for _ in range(30):   # phase B: isolated, real buffers
    gemm.decode_residual(e.c, e.dec_shadow, x, e.r, e.dec_part)
torch.cuda.synchronize()
for _ in range(30):
    gemm.encode_relu(x, e.enc_shadow, e.params["encoder_bias"], e.c, e.enc_part, None, None, mask_out=e.cmask)
torch.cuda.synchronize()
# phase C: dense random codes
c2 = torch.rand_like(e.c.float()).to(torch.bfloat16)
for _ in range(30):
    gemm.decode_residual(c2, e.dec_shadow, x, e.r, e.dec_part)
torch.cuda.synchronize()
# phase D: ENC -> DEC -> DEC (is the first DEC after ENC slow because c was just written?)
for _ in range(20):
    gemm.encode_relu(x, e.enc_shadow, e.params["encoder_bias"], e.c, e.enc_part, None, None, mask_out=e.cmask)
    gemm.decode_residual(e.c, e.dec_shadow, x, e.r, e.dec_part)
    gemm.decode_residual(e.c, e.dec_shadow, x, e.r, e.dec_part)
torch.cuda.synchronize()
print("done")
