"""UnrolledEnsemble on the grouped MFMA GEMM (bf16 operands, fp32 accumulation): every
parameter gradient of every model against the same engine's fp32 torch.matmul path (CPU),
per-model relative Frobenius error <= 3e-2 through 3 unrolled layers; one Adam step then
moves the parameters like the fp32 oracle."""

import pytest
import torch

from sparse_coding__amd.engine.unrolled import UnrolledEnsemble, _GroupedMM, grouped_mm
from sparse_coding__amd.models.lista import FunctionalLISTADenoisingSAE, FunctionalResidualDenoisingSAE

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("tb", [True, False])
@pytest.mark.parametrize("shared", [True, False])
def test_grouped_mm_kernel_forward_backward(tb, shared):
    torch.manual_seed(1)
    G, M, K, N = 3, 256, 128, 384
    a = torch.randn(*((M, K) if shared else (G, M, K)), device=DEV, requires_grad=True)
    b = torch.randn(*((G, N, K) if tb else (G, K, N)), device=DEV, requires_grad=True)
    out = _GroupedMM.apply(a, b, tb)
    g = torch.randn_like(out)
    da, db = torch.autograd.grad(out, [a, b], g)
    a32, b32 = a.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    ref = torch.matmul(a32.to(torch.bfloat16).float(), (b32.transpose(1, 2) if tb else b32).to(torch.bfloat16).float())
    ra, rb = torch.autograd.grad(ref, [a32, b32], g)
    assert _rel(out, ref) < 1e-4
    assert _rel(da, ra) < 1e-2 and _rel(db, rb) < 1e-2


@pytest.mark.parametrize("sig", [FunctionalLISTADenoisingSAE, FunctionalResidualDenoisingSAE])
def test_unrolled_hip_grads_match_fp32(sig):
    torch.manual_seed(2)
    d, n, B, G = 128, 256, 256, 3
    models = [sig.init(d, n, 3, l1) for l1 in (1e-3, 3e-3, 1e-2)]
    x = torch.randn(B, d)
    hip = UnrolledEnsemble(models, sig, device=DEV)
    ref = UnrolledEnsemble(models, sig, device="cpu")
    gh, (th, _, _, _) = hip.grads(x.to(DEV))
    gr, (tr, _, _, _) = ref.grads(x)
    torch.testing.assert_close(th.cpu(), tr, rtol=2e-2, atol=1e-4)
    for k in gr:
        for g in range(G):
            e = _rel(gh[k][g], gr[k][g])
            assert e <= 3e-2, (k, g, e)
    assert grouped_mm(x.to(DEV), hip.params["decoder"].detach(), tb=True).is_cuda
