"""Runs each kernel of the fused SAE step (config 2 shapes, as the engine launches them: the
code gradient from the encoder's activity mask, the fused step tail) a few times, plus the top-k
scores GEMM (bf16 out) and select of config 4 and a config-5 FISTA solve (d = n = 1024, 8 models, 20 iterations), for
rocprofv3 counter collection (scripts/gpu.sh pmc)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from sparse_coding__amd.engine.fused import FusedSAEEnsemble
from sparse_coding__amd.models.signatures import FunctionalSAE
from sparse_coding__amd.ops import adam as adam_ops
from sparse_coding__amd.ops import gemm
from sparse_coding__amd.ops import topk as topk_ops

B, d, n, G = 2048, 512, 2048, 8
dev = "cuda"
models = [FunctionalSAE.init(d, n, 1e-3 * (i + 1), device=dev) for i in range(G)]
e = FusedSAEEnsemble(models, FunctionalSAE, batch_size=B, device=dev)
x = (torch.randn(B, d, device=dev) * 0.4).to(torch.bfloat16)
for _ in range(3):
    e.step_batch(x)
torch.cuda.synchronize()
for _ in range(5):
    gemm.encode_relu(x, e.enc_shadow, e.params["encoder_bias"], e.c, e.enc_part, None, None, mask_out=e.cmask)
    gemm.decode_residual(e.c, e.dec_shadow, x, e.r, e.dec_part)
    gemm.code_grad(e.r, e.dec_shadow, e.c, e.l1, e.dpre, e.colpart, mask=e.cmask)
    gemm.weight_grads([[(e.c, e.r)], [(e.dpre, x)]], [e.g_dec, e.g_enc], 1e-6)
    e._apply_update_kernels()  # the fused step tail (row Adam + losses + bias Adam)
torch.cuda.synchronize()
# config 4 top-k: bf16 scores GEMM + select (8 models, B=2048, d=768, n=6144)
xt = (torch.randn(2048, 768, device=dev) * 0.3).to(torch.bfloat16)
Dt = torch.nn.functional.normalize(torch.randn(8, 6144, 768, device=dev), dim=-1).to(torch.bfloat16)
scores = torch.empty(8, 2048, 6144, device=dev, dtype=torch.bfloat16)
k = torch.tensor([8, 16, 24, 32, 48, 64, 96, 128], dtype=torch.int32, device=dev)
for _ in range(3):
    gemm.matmul_nt(xt, Dt, scores)
    topk_ops.topk_select(scores, k, 128, x=xt, D=Dt)
torch.cuda.synchronize()
# config 5 FISTA: Gram-form persistent solve, 8 models, d = n = 1024, B = 2048
from sparse_coding__amd.ops import fista as F  # noqa: E402

D = torch.nn.functional.normalize(torch.randn(8, 1024, 1024, device=dev), dim=-1)
X = torch.randn(2048, 1024, device=dev) * 0.1
lam = torch.full((8,), 1e-3, device=dev)
for _ in range(2):
    F.fista(X, D, lam, iters=20, backend="hip")
torch.cuda.synchronize()
print("done")
