"""Runs each fused-step kernel a few times (for rocprofv3 counter collection)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from sparse_coding__amd.engine.fused import FusedSAEEnsemble
from sparse_coding__amd.models.signatures import FunctionalSAE
from sparse_coding__amd.ops import gemm

B, d, n, G = 2048, 512, 2048, 8
dev = "cuda"
models = [FunctionalSAE.init(d, n, 1e-3 * (i + 1), device=dev) for i in range(G)]
e = FusedSAEEnsemble(models, FunctionalSAE, batch_size=B, device=dev)
x = torch.randn(B, d, device=dev).to(torch.bfloat16)
for _ in range(3):
    e.step_batch(x)
torch.cuda.synchronize()
for _ in range(5):
    gemm.encode_relu(x, e.enc_shadow, e.params["encoder_bias"], e.c, e.enc_part, e.cnt_part, None)
    gemm.decode_residual(e.c, e.dec_shadow, x, e.r, e.dec_part)
    gemm.code_grad(e.r, e.dec_shadow, e.c, e.l1, e.dpre, e.colpart)
    gemm.weight_grads([[(e.c, e.r)], [(e.dpre, x)]], [e.g_dec, e.g_enc], 1e-6)
torch.cuda.synchronize()
print("done")
