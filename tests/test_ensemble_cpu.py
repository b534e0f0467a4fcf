"""CPU tests of the oracle path: signatures, functional Adam, FunctionalEnsemble (config 1)."""

import numpy as np
import pytest
import torch

from sparse_coding__amd.data.synthetic import RandomDatasetGenerator
from sparse_coding__amd.engine.ensemble import FunctionalEnsemble, stack_dict, unstack_dict
from sparse_coding__amd.engine.optim import adam, sgd
from sparse_coding__amd.models import signatures as S
from sparse_coding__amd.models.learned_dict import TiedSAE, UntiedSAE


def test_stack_unstack_roundtrip():
    ms = [S.FunctionalSAE.init(8, 16, l1) for l1 in (1e-3, 2e-3)]
    p = stack_dict([m[0] for m in ms])
    assert p["encoder"].shape == (2, 16, 8)
    back = unstack_dict(p, 2)
    torch.testing.assert_close(back[1]["decoder"], ms[1][0]["decoder"])


def test_functional_adam_matches_torch_adam():
    torch.manual_seed(0)
    p = torch.randn(5, 7)
    opt = adam(lr=1e-2)
    st = opt.init({"w": p.clone()})
    params = {"w": p.clone()}
    tp = torch.nn.Parameter(p.clone())
    topt = torch.optim.Adam([tp], lr=1e-2, eps=1e-8)
    for _ in range(4):
        g = torch.randn(5, 7)
        upd, st = opt.update({"w": g}, st)
        params["w"] += upd["w"]
        tp.grad = g.clone()
        topt.step()
    torch.testing.assert_close(params["w"], tp.detach(), rtol=1e-5, atol=1e-6)


def test_vmap_grads_match_per_model_autograd():
    torch.manual_seed(1)
    models = [S.FunctionalSAE.init(16, 32, l1) for l1 in (1e-3, 1e-2)]
    ens = FunctionalEnsemble(models, S.FunctionalSAE, adam, {"lr": 1e-3}, device="cpu")
    x = torch.randn(64, 16)
    grads, (ld, aux) = ens.compute_grads(x)
    for i, (p, b) in enumerate(models):
        pp = {k: v.clone().requires_grad_() for k, v in p.items()}
        loss, _ = S.FunctionalSAE.loss(pp, b, x)
        loss.backward()
        for k in pp:
            torch.testing.assert_close(grads[k][i], pp[k].grad, rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(ld["loss"][i], loss.detach())


@pytest.mark.parametrize("sig", [S.FunctionalSAE, S.FunctionalTiedSAE, S.FunctionalReverseSAE,
                                 S.FunctionalTiedCenteredSAE, S.FunctionalThresholdingSAE])
def test_every_signature_trains(sig):
    torch.manual_seed(2)
    gen = RandomDatasetGenerator(32, 64, 256, 4, 0.99, False, "cpu", seed=0)
    models = [sig.init(32, 64, l1) for l1 in (1e-4, 1e-3)]
    ens = FunctionalEnsemble(models, sig, "adam", {"lr": 3e-3}, device="cpu")
    first = None
    for step in range(60):
        loss, _ = ens.step_batch(next(gen))
        first = loss["loss"].clone() if first is None else first
    assert (loss["loss"] < first).all(), (first, loss["loss"])
    lds = ens.to_learned_dicts()
    x = next(gen)
    for ld in lds:
        assert ld.predict(x).shape == x.shape
        assert ld.encode(x).shape == (256, 64)


def test_masked_signatures_respect_dict_size():
    torch.manual_seed(3)
    models = [S.FunctionalMaskedSAE.init(16, n, 64, 1e-3) for n in (16, 32, 64)]
    ens = FunctionalEnsemble(models, S.FunctionalMaskedSAE, adam, {"lr": 1e-3}, device="cpu")
    x = torch.randn(32, 16)
    _, (ld, aux) = ens.compute_grads(x)
    c = aux["c"]
    assert (c[0, :, 16:] == 0).all() and (c[1, :, 32:] == 0).all()
    lds = ens.to_learned_dicts()
    assert [ld.n_feats for ld in lds] == [16, 32, 64]


def test_config1_tied_sae_cpu_end_to_end():
    """BASELINE config 1: single tied SAE, d=128, ratio 2, l1=1e-3, on the random dataset."""
    torch.manual_seed(0)
    d, ratio = 128, 2
    gen = RandomDatasetGenerator(d, 256, 256, 8, 0.99, False, "cpu", seed=0)
    models = [S.FunctionalTiedSAE.init(d, d * ratio, 1e-3)]
    ens = FunctionalEnsemble(models, S.FunctionalTiedSAE, adam, {"lr": 1e-3}, device="cpu")
    losses = []
    for _ in range(300):
        loss, _ = ens.step_batch(next(gen))
        losses.append(float(loss["loss"][0]))
    assert losses[-1] < 0.5 * losses[0]
    ld = ens.to_learned_dicts()[0]
    assert isinstance(ld, TiedSAE) and ld.norm_encoder
    from sparse_coding__amd.eval.metrics import fraction_variance_unexplained, mean_l0, mmcs_to_fixed

    x = next(gen)
    assert float(fraction_variance_unexplained(ld, x)) < 0.5
    assert float(mean_l0(ld, x)) > 0
    assert float(mmcs_to_fixed(ld, gen.feats)) > 0.3


def test_sgd_optimizer_runs():
    models = [S.FunctionalSAE.init(8, 16, 1e-3)]
    ens = FunctionalEnsemble(models, S.FunctionalSAE, sgd, {"lr": 1e-2, "momentum": 0.9}, device="cpu")
    ens.step_batch(torch.randn(16, 8))


def _analytic_vs_autograd(sig, models, steps=3, lr=1e-3):
    import torch

    from sparse_coding__amd.engine.analytic import AnalyticSAEEnsemble
    from sparse_coding__amd.engine.ensemble import FunctionalEnsemble
    from sparse_coding__amd.engine.optim import adam

    clone = lambda ms: [({k: v.clone() for k, v in p.items()}, {k: v.clone() for k, v in b.items()}) for p, b in ms]
    ref = FunctionalEnsemble(clone(models), sig, adam, {"lr": lr})
    ana = AnalyticSAEEnsemble(clone(models), sig, lr=lr)
    g = torch.Generator().manual_seed(1)
    for _ in range(steps):
        x = torch.randn(64, models[0][0]["encoder"].shape[1], generator=g)
        lr_, _ = ref.step_batch(x)
        la, _ = ana.step_batch(x)
        for k in la:
            torch.testing.assert_close(la[k], lr_[k], rtol=1e-5, atol=1e-6)
    for k in ana.params:
        torch.testing.assert_close(ana.params[k], ref.params[k].detach(), rtol=1e-4, atol=1e-5)


def test_analytic_engine_matches_autograd_all_sae_kinds():
    import torch

    from sparse_coding__amd.models.signatures import (FunctionalMaskedSAE, FunctionalMaskedTiedSAE, FunctionalSAE,
                                                      FunctionalTiedSAE)

    torch.manual_seed(0)
    _analytic_vs_autograd(FunctionalSAE, [FunctionalSAE.init(16, 32, l1, bias_decay=bd)
                                          for l1, bd in ((1e-3, 0.0), (3e-3, 0.1))])
    rot = torch.linalg.qr(torch.randn(16, 16))[0]
    _analytic_vs_autograd(FunctionalTiedSAE, [FunctionalTiedSAE.init(16, 32, 1e-3, bias_decay=0.05, rotation=rot,
                                                                     translation=torch.randn(16),
                                                                     scaling=torch.rand(16) + 0.5)
                                              for _ in range(2)])
    _analytic_vs_autograd(FunctionalMaskedTiedSAE, [FunctionalMaskedTiedSAE.init(16, s, 32, 1e-3) for s in (16, 32)])
    _analytic_vs_autograd(FunctionalMaskedSAE, [FunctionalMaskedSAE.init(16, s, 32, 1e-3) for s in (8, 32)])


def test_debug_utilities():
    import pytest
    import torch

    from sparse_coding__amd.engine.analytic import AnalyticSAEEnsemble
    from sparse_coding__amd.models.signatures import FunctionalSAE
    from sparse_coding__amd.ops import _lib
    from sparse_coding__amd.utils import debug

    with debug.debug_mode():
        assert _lib._DEBUG_SYNC
    assert not _lib._DEBUG_SYNC
    debug.check_finite({"a": torch.ones(3)})
    with pytest.raises(FloatingPointError):
        debug.check_finite({"a": torch.tensor([1.0, float("nan")])}, "after step 3")
    x = torch.randn(32, 8)

    def make():
        torch.manual_seed(0)
        return AnalyticSAEEnsemble([FunctionalSAE.init(8, 16, 1e-3) for _ in range(2)], FunctionalSAE)

    def step(e):
        e.step_batch(x)
        return dict(e.params)

    debug.assert_deterministic(make, step)
    with debug.serialize_streams():
        import os

        assert os.environ["SC_SERIALIZE_STREAMS"] == "1"
