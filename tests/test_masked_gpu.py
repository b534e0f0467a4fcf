"""Masked ensembles (models of several live sizes stacked to one width, reference
autoencoders/sae_ensemble.py:306-442): the compacted launches -- only live tiles, nothing past a
model's live size written -- give the same results as the full masked launches."""

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from sparse_coding__amd.ops import _lib as L

    L.lib()  # must load: no silent fallback on a GPU box
    yield


@pytest.mark.parametrize("cfg", [1, 3])
def test_compacted_masked_launches_match_full(cfg):
    from sparse_coding__amd.ops import gemm

    torch.manual_seed(2)
    G, B, d, n = 4, 512, 256, 768
    sizes = [128, 300, 512, 768]
    live = torch.tensor(sizes, device=DEV, dtype=torch.int32)
    x = (torch.randn(B, d, device=DEV)).to(torch.bfloat16)
    we = (torch.randn(G, n, d, device=DEV) * 0.05).to(torch.bfloat16)
    wd = torch.nn.functional.normalize(torch.randn(G, n, d, device=DEV), dim=-1).to(torch.bfloat16)
    bias = torch.randn(G, n, device=DEV) * 0.1
    l1 = torch.tensor([1e-3, 2e-3, 3e-3, 4e-3], device=DEV)
    outs = {}
    with gemm.force_shape(cfg if cfg != 3 else 1):
        for mode, host in (("full", None), ("comp", sizes)):
            c = torch.zeros(G, B, n, device=DEV, dtype=torch.bfloat16) if host else \
                torch.full((G, B, n), 7.0, device=DEV, dtype=torch.bfloat16)
            part = torch.zeros(G, (B // 128) * (n // 128), 2, device=DEV)
            cnt = torch.zeros(G, B // 128, n, device=DEV)
            cmask = torch.zeros(gemm.code_mask_shape(G, B, n), device=DEV, dtype=torch.int64)
            gemm.encode_relu(x, we, bias, c, part, cnt, live, mask_out=cmask, live_host=host)
            r = torch.empty(G, B, d, device=DEV, dtype=torch.bfloat16)
            dpart = torch.zeros(G, (B // 128) * (d // 128), device=DEV)
            gemm.decode_residual(c, wd, x, r, dpart, nactive=live)
            dpre = torch.zeros(G, B, n, device=DEV, dtype=torch.bfloat16)
            colpart = torch.zeros(G, B // 128, n, device=DEV)
            gemm.code_grad(r, wd, c, l1, dpre, colpart, mask=cmask, nactive=live, live_host=host)
            outs[mode] = dict(c=c, part=part.sum(1), cnt=cnt, r=r, dpart=dpart.sum(1), dpre=dpre, colpart=colpart)
    with gemm.force_shape(cfg):
        for mode, host in (("full", None), ("comp", sizes)):
            o = outs[mode]
            gw = torch.zeros(2, G, n, d, device=DEV) if host else torch.full((2, G, n, d), 5.0, device=DEV)
            gemm.weight_grads([[(o["c"], o["r"])], [(o["dpre"], x)]], [gw[0], gw[1]], 0.5, nactive=live,
                              live_host=host)
            o["gw"] = gw
    torch.cuda.synchronize()
    f, c_ = outs["full"], outs["comp"]
    assert torch.equal(f["c"], c_["c"])                     # dead codes: zero in both
    assert torch.equal(f["r"], c_["r"])
    for g, s in enumerate(sizes):                           # dpre past dict_size: unwritten by design
        assert torch.equal(f["dpre"][g, :, :s], c_["dpre"][g, :, :s])
        assert not c_["dpre"][g, :, s:].any()
    torch.testing.assert_close(f["part"], c_["part"], rtol=0, atol=0)
    torch.testing.assert_close(f["cnt"], c_["cnt"], rtol=0, atol=0)
    torch.testing.assert_close(f["colpart"], c_["colpart"], rtol=0, atol=0)
    torch.testing.assert_close(f["dpart"], c_["dpart"], rtol=0, atol=0)
    assert torch.equal(f["gw"], c_["gw"])                   # dead gradient rows: zero in both


@pytest.mark.parametrize("kind", ["untied", "tied"])
def test_masked_engine_matches_eager(kind):
    from sparse_coding__amd.engine.ensemble import FunctionalEnsemble
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.engine.optim import adam
    from sparse_coding__amd.models.signatures import FunctionalMaskedSAE, FunctionalMaskedTiedSAE

    torch.manual_seed(6)
    sig = FunctionalMaskedSAE if kind == "untied" else FunctionalMaskedTiedSAE
    d, stack, B = 256, 768, 256
    sizes = [256, 384, 512, 768]
    models = [sig.init(d, s, stack, 1e-3, device=DEV) for s in sizes]
    ref = FunctionalEnsemble([({k: v.clone() for k, v in p.items()}, b) for p, b in models], sig, adam,
                             {"lr": 1e-3}, device=DEV)
    fused = FusedSAEEnsemble(models, sig, lr=1e-3, batch_size=B, device=DEV).enable_graph()
    feats = torch.nn.functional.normalize(torch.randn(1024, d, device=DEV), dim=-1)
    for _ in range(4):
        x = (torch.relu(torch.randn(B, 1024, device=DEV) - 2.0) @ feats).to(torch.bfloat16)
        loss_ref, _ = ref.step_batch(x.float())
        out = fused.step_batch(x)
        torch.cuda.synchronize()
        torch.testing.assert_close(out[:, 0], loss_ref["loss"], rtol=3e-2, atol=1e-4)
    for k in fused.params:
        if fused.params[k].dim() != 3:
            continue
        init = torch.stack([p[k] for p, _ in models])
        for g, s in enumerate(sizes):
            assert torch.equal(fused.params[k][g, s:], init[g, s:]), (k, g)
            mv_f = (fused.params[k][g, :s] - init[g, :s]).flatten()
            mv_r = (ref.params[k][g, :s] - init[g, :s]).flatten()
            assert torch.nn.functional.cosine_similarity(mv_f, mv_r, dim=0).item() > 0.97, (k, g)


def test_compacted_split_k_weight_gradient():
    """Split-K weight gradient on the compacted masked grid: the partial slabs sum to the unsplit
    product, and rows past each model's live size stay untouched."""
    from sparse_coding__amd.ops import gemm

    torch.manual_seed(3)
    G, B, n, d = 3, 2048, 768, 256
    sizes = [256, 500, 768]
    live = torch.tensor(sizes, device=DEV, dtype=torch.int32)
    c = torch.zeros(G, B, n, device=DEV, dtype=torch.bfloat16)
    for g, s in enumerate(sizes):
        c[g, :, :s] = torch.randn(B, s, device=DEV).to(torch.bfloat16)
    r = torch.randn(G, B, d, device=DEV).to(torch.bfloat16)
    ref = torch.zeros(G, n, d, device=DEV)
    gemm.weight_grads([[(c, r)]], [ref], 0.25, nactive=live, live_host=sizes)
    parts = torch.zeros(2, G, n, d, device=DEV)
    gemm.weight_grads([[(c, r)]], [parts], 0.25, ksplit=2, nactive=live, live_host=sizes)
    torch.cuda.synchronize()
    exp = 0.25 * c.float().transpose(1, 2) @ r.float()
    torch.testing.assert_close(ref, exp, rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(parts.sum(0), ref, rtol=1e-4, atol=1e-3)
    for g, s in enumerate(sizes):
        assert not parts[:, g, s:].any() and not ref[g, s:].any()

