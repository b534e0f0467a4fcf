"""FISTA-in-the-loss (reference autoencoders/fista.py:141-172): the explicit adjoint of the
unrolled solver against autograd through every iteration, and the ensemble engine's gradients
against per-model autograd of the loss2 objective."""
import torch

from sparse_coding__amd.ops import fista as F


def _autograd_unrolled(X, D, lam, A0, iters, eta):
    mom = F.momentum_schedule(iters).tolist()
    A = Y = A0
    for t in range(iters):
        A_prev = A
        Y = Y + eta * (X - Y @ D) @ D.T
        A = torch.clamp(Y - eta * lam, min=0.0)
        Y = A + (A - A_prev) * mom[t]
    return X - A @ D


def test_unrolled_fista_adjoint_matches_autograd():
    torch.manual_seed(0)
    G, B, n, d, T = 3, 16, 48, 24, 15
    D = torch.nn.functional.normalize(torch.randn(G, n, d, dtype=torch.float64), dim=-1).float()
    X = torch.randn(B, d)
    c = torch.relu(torch.randn(G, B, n)) * 0.1
    lam = torch.tensor([1e-3, 1e-2, 3e-2])
    eta = F.step_size(D)
    W = torch.randn(G, B, d)
    D1, c1 = D.clone().requires_grad_(), c.clone().requires_grad_()
    R = F.unrolled_fista_residual(X, D1, lam, c1, T, eta, backend="torch")
    (R * W).sum().backward()
    for g in range(G):
        D2, c2 = D[g].clone().requires_grad_(), c[g].clone().requires_grad_()
        R2 = _autograd_unrolled(X, D2, lam[g], c2, T, eta[g])
        (R2 * W[g]).sum().backward()
        torch.testing.assert_close(R[g], R2, rtol=1e-5, atol=1e-5)
        assert (D1.grad[g] - D2.grad).norm() / D2.grad.norm() < 1e-5
        assert (c1.grad[g] - c2.grad).norm() / c2.grad.norm() < 1e-5


def test_loss2_uses_adjoint_and_matches_reference_formula():
    from sparse_coding__amd.models.fista import FunctionalFista

    torch.manual_seed(1)
    p, b = FunctionalFista.init(16, 32, 1e-3)
    x = torch.randn(24, 16)
    pr = {k: v.clone().requires_grad_() for k, v in p.items()}
    loss, _ = FunctionalFista.loss2(pr, b, x, num_iter=8)
    loss.backward()
    # reference formula through plain autograd
    pq = {k: v.clone().requires_grad_() for k, v in p.items()}
    w = pq["encoder"] / pq["encoder"].norm(dim=-1, keepdim=True)
    c = torch.relu(x @ w.T + pq["encoder_bias"])
    # upstream (autoencoders/fista.py:104-106) does NOT detach eta: its gradient path counts
    eta = 1.0 / torch.linalg.eigvalsh(w @ w.T).max()
    ref = ((c @ w - x).pow(2).mean() + b["l1_alpha"] * c.abs().sum(-1).mean()
           + _autograd_unrolled(x, w, b["l1_alpha"], c, 8, eta).pow(2).mean())
    ref.backward()
    torch.testing.assert_close(loss.detach(), ref.detach(), rtol=1e-5, atol=1e-6)
    for k in ("encoder", "encoder_bias"):
        torch.testing.assert_close(pr[k].grad, pq[k].grad, rtol=1e-4, atol=1e-6)


def test_unrolled_eta_gradient_matches_autograd():
    """dL/deta of the explicit adjoint (sum_t <S_t, Res_t> - lam sum Vbar_t) against autograd
    through every iteration."""
    torch.manual_seed(5)
    G, B, n, d, T = 2, 12, 32, 16, 9
    D = torch.nn.functional.normalize(torch.randn(G, n, d), dim=-1)
    X = torch.randn(B, d)
    c = torch.relu(torch.randn(G, B, n)) * 0.1
    lam = torch.tensor([1e-3, 2e-2])
    eta = F.step_size(D).clone().requires_grad_()
    W = torch.randn(G, B, d)
    (F.unrolled_fista_residual(X, D, lam, c, T, eta, backend="torch") * W).sum().backward()
    for g in range(G):
        e2 = eta.detach()[g].clone().requires_grad_()
        (_autograd_unrolled(X, D[g], lam[g], c[g], T, e2) * W[g]).sum().backward()
        torch.testing.assert_close(eta.grad[g], e2.grad, rtol=1e-4, atol=1e-5)


def test_loss2_under_vmap_grad_matches_per_model_autograd():
    """FunctionalFista.loss2 keeps working under functorch (vmap(grad(loss)) of the eager
    ensemble): the iterations then run as plain differentiable ops."""
    from torch.func import grad, vmap

    from sparse_coding__amd.models.fista import FunctionalFista

    torch.manual_seed(6)
    models = [FunctionalFista.init(16, 32, l1) for l1 in (1e-3, 1e-2)]
    x = torch.randn(20, 16)
    params = {k: torch.stack([m[0][k] for m in models]) for k in ("encoder", "encoder_bias")}
    bufs = {"l1_alpha": torch.tensor([m[1]["l1_alpha"] for m in models])}

    def loss(p, b):
        return FunctionalFista.loss2(p, b, x, num_iter=6)[0]

    gv = vmap(grad(loss))(params, bufs)
    for g, (p, b) in enumerate(models):
        pq = {k: p[k].clone().requires_grad_() for k in ("encoder", "encoder_bias")}
        FunctionalFista.loss2(pq, b, x, num_iter=6)[0].backward()
        for k in pq:
            torch.testing.assert_close(gv[k][g], pq[k].grad, rtol=1e-4, atol=1e-6)


def test_fista_loss_ensemble_gradients_cpu():
    from sparse_coding__amd.engine.fista_loss import FistaLossEnsemble
    from sparse_coding__amd.models.fista import FunctionalFista

    torch.manual_seed(2)
    d, n, B, T = 16, 32, 24, 6
    models = [FunctionalFista.init(d, n, l1) for l1 in (1e-4, 1e-3, 1e-2)]
    eng = FistaLossEnsemble(models, lr=1e-3, batch_size=B, device="cpu", num_iter=T)
    x = torch.randn(B, d)
    total, _ = eng.losses(x)  # the tracker's first call is an exact eigh
    total.sum().backward()
    for g, (p, b) in enumerate(models):
        pq = {k: v.clone().requires_grad_() for k, v in p.items()}
        w = pq["encoder"] / pq["encoder"].norm(dim=-1, keepdim=True)
        c = torch.relu(x @ w.T + pq["encoder_bias"])
        eta = 1.0 / torch.linalg.eigvalsh(w @ w.T).max()  # differentiable, as upstream
        ref = ((c @ w - x).pow(2).mean() + b["l1_alpha"] * c.abs().sum(-1).mean()
               + _autograd_unrolled(x, w, b["l1_alpha"], c, T, eta).pow(2).mean())
        ref.backward()
        torch.testing.assert_close(total[g].detach(), ref.detach(), rtol=1e-5, atol=1e-6)
        for k in ("encoder", "encoder_bias"):
            got = eng.params[k].grad[g]
            assert (got - pq[k].grad).norm() / pq[k].grad.norm() < 1e-4, k
    before = eng.params["encoder"].detach().clone()
    eng.opt.step()
    assert not torch.equal(before, eng.params["encoder"].detach())


def test_trainer_fista_loss_objective_cpu(tmp_path):
    from sparse_coding__amd.engine.trainer import EnsembleTrainer
    from sparse_coding__amd.models.fista import FunctionalFista

    torch.manual_seed(3)
    d, n, B = 16, 32, 24
    models = [FunctionalFista.init(d, n, l1) for l1 in (1e-4, 1e-2)]
    tr = EnsembleTrainer(models, FunctionalFista, lr=1e-2, batch_size=B, device="cpu", objective="fista_loss",
                         fista_loss_iters=5)
    assert tr.kind == "fista-loss" and tr.fista is None
    x = torch.randn(B, d)
    first = tr.step(x).clone()
    for _ in range(30):
        last = tr.step(x)
    assert (last < first).all()
    hosts = tr.losses_host()
    assert set(hosts[0]) >= {"loss", "l_reconstruction", "l_fista", "l_l1"}
    lds = tr.to_learned_dicts(ensemble_hyperparams=())
    assert len(lds) == 2 and lds[0][0].get_learned_dict().shape == (n, d)
    st = tr.state_dict()
    tr2 = EnsembleTrainer(models, FunctionalFista, lr=1e-2, batch_size=B, device="cpu", objective="fista_loss",
                          fista_loss_iters=5)
    tr2.load_state_dict(st)
    torch.testing.assert_close(tr2.impl.params["encoder"], tr.impl.params["encoder"])


def test_coef_search_torch_matches_basis_pursuit():
    from sparse_coding__amd.models.misc import DirectCoefOptimizer
    from sparse_coding__amd.models.signatures import unit_rows

    torch.manual_seed(4)
    p, b = DirectCoefOptimizer.init(16, 32, 1e-2, lr=1e-1)
    x = torch.randn(20, 16)
    with torch.no_grad():
        ref = DirectCoefOptimizer.basis_pursuit(p, b, x, n_iters=30)
        got = F.coef_search_torch(x, unit_rows(p["decoder"])[None], b["l1_alpha"], b["lr"], 30)[0]
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6)
