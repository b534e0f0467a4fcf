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


def test_lista_step_kernel_matches_torch_autograd():
    from sparse_coding__amd.engine.unrolled import _ListaStep
    from sparse_coding__amd.models.lista import shrinkage

    torch.manual_seed(5)
    G, B, n = 3, 128, 512
    y, a, xs = (torch.randn(G, B, n, device=DEV, requires_grad=True) for _ in range(3))
    theta = (torch.randn(G, n, device=DEV) * 0.3).requires_grad_()
    m = torch.tensor([0.1, 0.5, 0.9], device=DEV, requires_grad=True)
    yo, xo = _ListaStep.apply(y, a, xs, theta, m)
    x_ = shrinkage(y + a, theta.unsqueeze(1))
    yr = x_ + m.view(-1, 1, 1) * (x_ - xs)
    torch.testing.assert_close(yo, yr)
    torch.testing.assert_close(xo, x_)
    gy, gx = torch.randn_like(yo), torch.randn_like(xo)
    got = torch.autograd.grad([yo, xo], [y, a, xs, theta, m], [gy, gx])
    ref = torch.autograd.grad([yr, x_], [y, a, xs, theta, m], [gy, gx], retain_graph=True)
    for gg, rr in zip(got, ref):
        torch.testing.assert_close(gg, rr, rtol=1e-4, atol=1e-3)
    got1 = torch.autograd.grad(_ListaStep.apply(y, a, xs, theta, m)[0], [theta, m], gy)  # x_ unused
    ref1 = torch.autograd.grad(yr, [theta, m], gy)
    for gg, rr in zip(got1, ref1):
        torch.testing.assert_close(gg, rr, rtol=1e-4, atol=1e-3)


def test_unrolled_adam_kernel_matches_torch_adam():
    """The engine's Adam (row-Adam kernel for the matrices, torch for vectors) == torchopt Adam
    in torch on the same gradients, over two steps."""
    torch.manual_seed(6)
    d, n, B = 256, 256, 256
    models = [FunctionalLISTADenoisingSAE.init(d, n, 2, l1) for l1 in (1e-3, 1e-2)]
    eng = UnrolledEnsemble(models, FunctionalLISTADenoisingSAE, lr=1e-3, device=DEV)
    p = {k: v.detach().clone() for k, v in eng.params.items()}
    m = {k: torch.zeros_like(v) for k, v in p.items()}
    v_ = {k: torch.zeros_like(v) for k, v in p.items()}
    for t in (1, 2):
        grads, _ = eng.grads(torch.randn(B, d, device=DEV))
        eng.apply_grads(grads)
        for k in p:
            g = grads[k]
            m[k] = 0.9 * m[k] + 0.1 * g
            v_[k] = 0.999 * v_[k] + 0.001 * g * g
            lr = eng.lr.view(-1, *([1] * (p[k].dim() - 1)))
            p[k] = p[k] - lr * (m[k] / (1 - 0.9 ** t)) / ((v_[k] / (1 - 0.999 ** t)).sqrt() + 1e-8)
    torch.cuda.synchronize()
    for k in p:
        torch.testing.assert_close(eng.params[k].detach(), p[k], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("sig", [FunctionalLISTADenoisingSAE, FunctionalResidualDenoisingSAE])
@pytest.mark.parametrize("layers,n,B", [(3, 512, 256), (2, 768, 384), (1, 256, 128)])
def test_lista_fused_grads_match_fp32(layers, n, B, sig):
    """The explicit (autograd-free) LISTA / residual-denoising step's gradients == the engine's fp32
    torch path (CPU),
    every parameter of every model, per-model relative Frobenius error <= 3e-2 (or within 1.5x of the
    autograd GPU path's own distance, at the small shapes), losses alike (odd and even layer counts:
    paired and lone weight-gradient problems)."""
    torch.manual_seed(3)
    d, G = 256, 3
    models = [sig.init(d, n, layers, l1) for l1 in (1e-3, 3e-3, 1e-2)]
    for p_, _ in models:  # off the orthogonal init, where y_0 D reproduces x and the residual is ~0
        p_["decoder"] = p_["decoder"] + 0.3 * torch.randn_like(p_["decoder"]) / d ** 0.5
    x = torch.randn(B, d)
    hip = UnrolledEnsemble(models, sig, device=DEV)
    ref = UnrolledEnsemble(models, sig, device="cpu")
    assert hip._fused_ok(B)
    gh, (th, lh, l1h, ch) = hip.fused_grads(x.to(DEV))
    gr, (tr, lr_, l1r, cr) = ref.grads(x)
    torch.testing.assert_close(lh.cpu(), lr_, rtol=2e-2, atol=1e-5)
    torch.testing.assert_close(l1h.cpu(), l1r, rtol=2e-2, atol=1e-6)
    assert _rel(ch, cr) < 2e-2
    assert set(gh) == set(gr)
    ga, _ = hip.grads(x.to(DEV))  # the autograd path on the same bf16 kernels: its distance is the noise floor
    for k in gr:
        for g in range(G):
            e, ea = _rel(gh[k][g], gr[k][g]), _rel(ga[k][g], gr[k][g])
            assert e <= max(3e-2, 1.5 * ea), (k, g, e, ea)


@pytest.mark.parametrize("sig", [FunctionalLISTADenoisingSAE, FunctionalResidualDenoisingSAE])
def test_lista_fused_step_tracks_autograd_step(sig):
    """Three explicit steps (row Adam + bf16 shadows) move every parameter as close to three steps of
    the fp32 CPU path as three steps of the autograd GPU path do (Adam's early steps are sign-like,
    so near-zero gradient entries flip either way); the maintained decoder shadow is the normalised
    decoder."""
    torch.manual_seed(4)
    d, n, B = 256, 512, 256
    models = [sig.init(d, n, 3, l1) for l1 in (1e-3, 1e-2)]
    fused = UnrolledEnsemble(models, sig, lr=1e-3, device=DEV)
    auto = UnrolledEnsemble(models, sig, lr=1e-3, device=DEV)
    ref = UnrolledEnsemble(models, sig, lr=1e-3, device="cpu")
    p0 = {k: v.detach().cpu().clone() for k, v in ref.params.items()}
    for _ in range(3):
        xb = torch.randn(B, d)
        out_f, _ = fused.step_batch(xb.to(DEV))
        g, _ = auto.grads(xb.to(DEV))
        auto.apply_grads(g)
        ref.step_batch(xb)
    torch.cuda.synchronize()
    for k in p0:
        dr = ref.params[k].detach() - p0[k]
        e_f = _rel(fused.params[k].cpu() - p0[k], dr)
        e_a = _rel(auto.params[k].cpu() - p0[k], dr)
        assert e_f <= max(1.5 * e_a, 2e-2), (k, e_f, e_a)
    dec = fused.params["decoder"].detach()
    want = (dec / dec.norm(dim=-1, keepdim=True)).to(torch.bfloat16).float()
    torch.testing.assert_close(fused._sh["decoder"].float(), want, rtol=1e-2, atol=1e-2)
    assert torch.isfinite(out_f["loss"]).all()


def test_lista_fused_training_and_resume():
    """The explicit LISTA step trains (loss falls over 60 steps) and resumes: a state_dict round trip
    into a fresh engine (bf16 shadows rebuilt from the loaded masters, which the running engine's Adam
    wrote itself -- the row norm may differ in the last bit) gives the same next step."""
    torch.manual_seed(8)
    d, n, B = 256, 512, 256
    sig = FunctionalLISTADenoisingSAE
    models = [sig.init(d, n, 2, l1) for l1 in (1e-4, 1e-3)]
    eng = UnrolledEnsemble(models, sig, lr=3e-3, device=DEV)
    basis = torch.randn(64, d, device=DEV)
    data = [(torch.rand(B, 64, device=DEV) ** 4) @ basis for _ in range(8)]
    first = last = None
    for t in range(60):
        out, _ = eng.step_batch(data[t % 8])
        if t == 0:
            first = out["l_reconstruction"].clone()
        last = out["l_reconstruction"]
    assert (last < 0.5 * first).all(), (first, last)
    sd = {k: ({kk: vv.clone() for kk, vv in v.items()} if isinstance(v, dict) else v) for k, v in eng.state_dict().items()}
    other = UnrolledEnsemble([sig.init(d, n, 2, l1) for l1 in (1e-4, 1e-3)], sig, lr=3e-3, device=DEV)
    other.load_state_dict(sd)
    a, _ = eng.step_batch(data[0])
    b, _ = other.step_batch(data[0])
    torch.cuda.synchronize()
    torch.testing.assert_close(a["loss"], b["loss"], rtol=1e-4, atol=1e-7)
    for k in eng.params:
        torch.testing.assert_close(eng.params[k], other.params[k], rtol=1e-4, atol=1e-6)
