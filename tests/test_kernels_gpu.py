"""Numerics of the gfx950 HIP kernels against plain PyTorch fp32 references."""

import io

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from sparse_coding__amd.ops import _lib as L

    L.lib()  # must load: no silent fallback on a GPU box
    yield


def _bf(*shape, scale=1.0, gen=None):
    return (torch.randn(*shape, device=DEV, generator=gen) * scale).to(torch.bfloat16)


def _close(a, b, rtol=2e-2, atol=1e-2):
    a = a.float()
    b = b.float()
    err = (a - b).abs().max().item()
    ref = b.abs().max().item()
    assert err <= atol + rtol * ref, f"max err {err} vs ref scale {ref}"


SHAPE_CFGS = [1, 2, 3]  # 128x128, 256x128, 256x256 blocks


@pytest.mark.parametrize("cfg", SHAPE_CFGS)
@pytest.mark.parametrize("G,M,N,K", [(1, 128, 128, 64), (3, 256, 384, 192), (2, 512, 256, 512), (2, 256, 512, 128)])
def test_matmul_layouts(G, M, N, K, cfg):
    from sparse_coding__amd.ops import gemm

    if not gemm.shape_fits(cfg, M, N):
        pytest.skip("block shape does not tile this problem")
    with gemm.force_shape(cfg):
        _matmul_layouts(G, M, N, K)


def _matmul_layouts(G, M, N, K):
    from sparse_coding__amd.ops import gemm

    torch.manual_seed(0)
    a = _bf(G, M, K)
    b = _bf(G, N, K)
    out = torch.empty(G, M, N, device=DEV)
    gemm.matmul_nt(a, b, out)
    _close(out, a.float() @ b.float().transpose(1, 2), rtol=1e-3, atol=1e-3)

    bn = _bf(G, K, N)
    gemm.matmul_nn(a, bn, out)
    _close(out, a.float() @ bn.float(), rtol=1e-3, atol=1e-3)

    at = _bf(G, K, M)
    gemm.matmul_tn(at, bn, out, alpha=0.5)
    _close(out, 0.5 * at.float().transpose(1, 2) @ bn.float(), rtol=1e-3, atol=1e-3)

    out16 = torch.empty(G, M, N, device=DEV, dtype=torch.bfloat16)
    gemm.matmul_nt(a, b, out16)
    _close(out16, a.float() @ b.float().transpose(1, 2), rtol=1e-2, atol=1e-2)


def test_identity_asymmetric():
    """A = I with an asymmetric B catches a transposed C write."""
    from sparse_coding__amd.ops import gemm

    M = K = 128
    N = 256
    a = torch.eye(M, K, device=DEV).to(torch.bfloat16)[None]
    b = torch.arange(N * K, device=DEV, dtype=torch.float32).reshape(1, N, K).remainder(97).to(torch.bfloat16)
    out = torch.empty(1, M, N, device=DEV)
    gemm.matmul_nt(a, b, out)
    torch.testing.assert_close(out, b.float().transpose(1, 2)[:, :M, :], rtol=0, atol=0)
    bt = b.transpose(1, 2).contiguous()  # [1, K, N]
    gemm.matmul_nn(a, bt, out)
    torch.testing.assert_close(out, bt.float()[:, :M, :], rtol=0, atol=0)
    gemm.matmul_tn(a, bt, out)
    torch.testing.assert_close(out, bt.float()[:, :M, :], rtol=0, atol=0)


PIPE_CFGS = [1 | 1 << 2, 1 | 2 << 2, 1 | 3 << 2, 3 | 1 << 2, 3 | 2 << 2, 3 | 3 << 2,  # deeper K pipelines
             1 | 2 << 2 | 16, 1 | 3 << 2 | 16,  # 128x128 BK32 rings, software-pipelined K loop
             2 | 3 << 2]  # 256x128 as eight 64x64 waves on BK32 x 3 (the encoder / masked code-gradient default)


@pytest.mark.parametrize("cfg", SHAPE_CFGS + PIPE_CFGS)
def test_sae_epilogues(cfg):
    from sparse_coding__amd.ops import gemm

    with gemm.force_shape(cfg):
        _sae_epilogues(3, 512, 256, 512 if cfg != 1 else 384)


def _sae_epilogues(G, B, d, n):
    from sparse_coding__amd.ops import gemm

    torch.manual_seed(1)
    x = _bf(B, d)
    we = _bf(G, n, d, scale=0.05)
    wd = torch.nn.functional.normalize(torch.randn(G, n, d, device=DEV), dim=-1).to(torch.bfloat16)
    bias = torch.randn(G, n, device=DEV) * 0.1
    nactive = torch.tensor([n, 256, 128], device=DEV, dtype=torch.int32)
    c = torch.empty(G, B, n, device=DEV, dtype=torch.bfloat16)
    part = torch.zeros(G, (B // 128) * (n // 128), 2, device=DEV)
    cnt = torch.zeros(G, B // 128, n, device=DEV)
    cmask = torch.zeros(gemm.code_mask_shape(G, B, n), device=DEV, dtype=torch.int64)
    gemm.encode_relu(x, we, bias, c, part, cnt, nactive, mask_out=cmask)
    ref = torch.relu(x.float() @ we.float().transpose(1, 2) + bias[:, None, :])
    for g in range(G):
        ref[g, :, int(nactive[g]):] = 0
    _close(c, ref)
    cf = c.float()
    torch.testing.assert_close(part[..., 0].sum(1), ref.sum((1, 2)), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(part[..., 1].sum(1), (cf > 0).float().sum((1, 2)), rtol=0, atol=0)
    torch.testing.assert_close(cnt.sum(1), (cf > 0).float().sum(1), rtol=0, atol=0)

    r = torch.empty(G, B, d, device=DEV, dtype=torch.bfloat16)
    dpart = torch.zeros(G, (B // 128) * (d // 128), device=DEV)
    gemm.decode_residual(c, wd, x, r, dpart)
    rref = cf @ wd.float() - x.float()
    _close(r, rref)
    torch.testing.assert_close(dpart.sum(1), (rref ** 2).sum((1, 2)), rtol=2e-2, atol=1e-1)

    l1 = torch.tensor([1e-3, 3e-3, 1e-2], device=DEV)
    dpre = torch.empty(G, B, n, device=DEV, dtype=torch.bfloat16)
    colpart = torch.zeros(G, B // 128, n, device=DEV)
    gemm.code_grad(r, wd, c, l1, dpre, colpart)
    dref = (r.float() @ wd.float().transpose(1, 2) + (l1 * d / 2)[:, None, None]) * (cf > 0)
    _close(dpre, dref)
    # bias-gradient partials are accumulated from the unrounded fp32 values
    _close(colpart.sum(1), dref.sum(1), rtol=1e-2, atol=1e-2)
    # the bitmask path (activity read from the encoder's ballots) is bit-identical
    dpre_m = torch.empty_like(dpre)
    colpart_m = torch.zeros_like(colpart)
    gemm.code_grad(r, wd, c, l1, dpre_m, colpart_m, mask=cmask)
    assert torch.equal(dpre_m, dpre)
    assert torch.equal(colpart_m, colpart)

    gd = torch.empty(G, n, d, device=DEV)
    ge = torch.empty(G, n, d, device=DEV)
    alpha = 2.0 / (B * d)
    gemm.weight_grads([[(c, r)], [(dpre, x)]], [gd, ge], alpha)
    _close(gd, alpha * cf.transpose(1, 2) @ r.float(), rtol=1e-3, atol=1e-6)
    _close(ge, alpha * dpre.float().transpose(1, 2) @ x.float(), rtol=1e-3, atol=1e-6)
    gt = torch.empty(G, n, d, device=DEV)
    gemm.weight_grads([[(c, r), (dpre, x)]], [gt], alpha)
    _close(gt, gd + ge, rtol=1e-3, atol=1e-6)


@pytest.mark.parametrize("cfg", [1 | 2 << 2, 1 | 3 << 2, 1 | 2 << 2 | 16, 1 | 3 << 2 | 16])
def test_bf16_epilogue_on_bk32_rings(cfg):
    """The plain bf16 epilogue on the 128x128 BK32 rings in the two top-k layouts: scores x D^T (both
    operands K-major) and the two-segment weight gradient codes^T R + dscore^T x (both M/N-major)."""
    from sparse_coding__amd.ops import gemm

    torch.manual_seed(21)
    G, B, n, d = 2, 256, 512, 768
    x, D = _bf(B, d), _bf(G, n, d)
    c, r, s = _bf(G, B, n), _bf(G, B, d), _bf(G, B, n)
    out = torch.empty(G, B, n, device=DEV, dtype=torch.bfloat16)
    g = torch.empty(G, n, d, device=DEV, dtype=torch.bfloat16)
    with gemm.force_shape(cfg):
        gemm.matmul_nt(x, D, out)
        gemm.weight_grads([[(c, r), (s, x)]], [g], 0.5)
    _close(out, x.float() @ D.float().transpose(1, 2), rtol=1e-2, atol=1e-2)
    ref = 0.5 * (c.float().transpose(1, 2) @ r.float() + s.float().transpose(1, 2) @ x.float())
    _close(g, ref, rtol=1e-2, atol=1e-2)


def test_adam_rows_matches_autograd():
    from sparse_coding__amd.ops import adam as adam_ops

    torch.manual_seed(2)
    G, n, d = 2, 128, 512
    p = torch.randn(G, n, d, device=DEV)
    p[0, 3] = 0.0  # exercise the 1e-8 clamp branch
    g_hat = torch.randn(G, n, d, device=DEV) * 1e-3
    m = torch.randn(G, n, d, device=DEV).abs() * 1e-4
    v = torch.randn(G, n, d, device=DEV).abs() * 1e-6
    lr = torch.tensor([1e-3, 2e-3], device=DEV)
    step = 5
    # reference: gradient through p / clamp(|p|, 1e-8) via autograd
    pr = p.clone().requires_grad_()
    w_hat = pr / torch.clamp(pr.norm(dim=-1, keepdim=True), min=1e-8)
    (w_hat * g_hat).sum().backward()
    g = pr.grad
    b1, b2, eps = 0.9, 0.999, 1e-8
    m_ref = b1 * m + (1 - b1) * g
    v_ref = b2 * v + (1 - b2) * g * g
    p_ref = p - lr[:, None, None] * (m_ref / (1 - b1 ** step)) / (torch.sqrt(v_ref / (1 - b2 ** step)) + eps)
    shadow = torch.empty(G, n, d, device=DEV, dtype=torch.bfloat16)
    p2, m2, v2 = p.clone(), m.clone(), v.clone()
    adam_ops.adam_rows([dict(p=p2, g=g_hat, m=m2, v=v2, shadow=shadow, norm=True)], lr, step, b1, b2, eps)
    torch.testing.assert_close(m2, m_ref, rtol=1e-4, atol=1e-9)
    torch.testing.assert_close(v2, v_ref, rtol=1e-4, atol=1e-12)
    torch.testing.assert_close(p2, p_ref, rtol=1e-4, atol=1e-6)
    sh_ref = p_ref / torch.clamp(p_ref.norm(dim=-1, keepdim=True), min=1e-8)
    _close(shadow, sh_ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("d", [512, 768])
def test_adam_rows_bf16_gradient_matches_fp32_kernel(d):
    """bf16-gradient Adam == the fp32-gradient kernel fed the same (bf16-rounded) gradient,
    including the split-K slab sum; the update arithmetic is fp32 in both."""
    from sparse_coding__amd.ops import adam as adam_ops

    torch.manual_seed(4)
    G, n = 3, 256
    p = torch.randn(G, n, d, device=DEV)
    gb = (torch.randn(2, G, n, d, device=DEV) * 1e-3).to(torch.bfloat16)
    m = torch.randn(G, n, d, device=DEV).abs() * 1e-4
    v = torch.randn(G, n, d, device=DEV).abs() * 1e-6
    lr = torch.tensor([1e-3, 2e-3, 5e-4], device=DEV)
    for nsplit in (1, 2):
        outs = []
        for g in (gb, gb.float()):
            st = dict(p=p.clone(), g=g[0], m=m.clone(), v=v.clone(),
                      shadow=torch.empty(G, n, d, device=DEV, dtype=torch.bfloat16),
                      norms=torch.empty(G, n, device=DEV), norm=True)
            adam_ops.adam_rows([st], lr, 7, nsplit=nsplit, gstride=G * n * d)
            outs.append(st)
        a, b = outs
        for k in ("p", "m", "v", "norms"):
            torch.testing.assert_close(a[k], b[k], rtol=1e-6, atol=1e-12)
        assert torch.equal(a["shadow"], b["shadow"])


def test_weight_grads_bf16_out_matches_fp32():
    from sparse_coding__amd.ops import gemm

    torch.manual_seed(5)
    G, Bk, n, d = 3, 1024, 512, 512
    A = (torch.randn(G, Bk, n, device=DEV) * 0.1).to(torch.bfloat16)
    Bm = (torch.randn(G, Bk, d, device=DEV) * 0.1).to(torch.bfloat16)
    A2 = (torch.randn(G, Bk, n, device=DEV) * 0.1).to(torch.bfloat16)
    for cfg in (1, 3):
        with gemm.force_shape(cfg):
            o32 = torch.empty(G, n, d, device=DEV)
            o16 = torch.empty(G, n, d, device=DEV, dtype=torch.bfloat16)
            gemm.weight_grads([[(A, Bm), (A2, Bm)]], [o32], 0.5)
            gemm.weight_grads([[(A, Bm), (A2, Bm)]], [o16], 0.5)
        torch.cuda.synchronize()
        ref = 0.5 * (A.float().transpose(1, 2) @ Bm.float() + A2.float().transpose(1, 2) @ Bm.float())
        torch.testing.assert_close(o32, ref, rtol=1e-3, atol=1e-3)
        assert torch.equal(o16, o32.to(torch.bfloat16)), cfg


@pytest.mark.parametrize("cfg", SHAPE_CFGS + [1 | 3 << 2 | 16])
@pytest.mark.parametrize("kind", ["untied", "tied"])
def test_fused_step_matches_functional_ensemble(kind, cfg):
    from sparse_coding__amd.ops import gemm

    with gemm.force_shape(cfg):
        _fused_step_matches(kind)


def _fused_step_matches(kind):
    from sparse_coding__amd.engine.ensemble import FunctionalEnsemble
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.engine.optim import adam
    from sparse_coding__amd.models.signatures import FunctionalSAE, FunctionalTiedSAE

    torch.manual_seed(3)
    sig = FunctionalSAE if kind == "untied" else FunctionalTiedSAE
    d, n, B, G = 256, 512, 256, 3
    l1s = [1e-4, 1e-3, 1e-2]
    models = [sig.init(d, n, l1, device=DEV) for l1 in l1s]
    ref = FunctionalEnsemble([({k: v.clone() for k, v in p.items()}, b) for p, b in models], sig, adam,
                             {"lr": 1e-3}, device=DEV)
    fused = FusedSAEEnsemble(models, sig, lr=1e-3, batch_size=B, device=DEV)
    feats = torch.nn.functional.normalize(torch.randn(1024, d, device=DEV), dim=-1)
    for step in range(5):
        codes = torch.relu(torch.randn(B, 1024, device=DEV) - 2.0)
        x = (codes @ feats).to(torch.bfloat16)
        loss_ref, _ = ref.step_batch(x.float())
        out = fused.step_batch(x)
        torch.cuda.synchronize()
        torch.testing.assert_close(out[:, 0], loss_ref["loss"], rtol=3e-2, atol=1e-4)
        torch.testing.assert_close(out[:, 1], loss_ref["l_reconstruction"], rtol=3e-2, atol=1e-4)
        torch.testing.assert_close(out[:, 2], loss_ref["l_l1"], rtol=3e-2, atol=1e-5)
        if step == 0:
            # gradient level: after one step Adam's first moment is (1 - b1) * g in both engines;
            # per model relative Frobenius error (the oracle runs fp32 weights, the kernels the
            # bf16-rounded encoder: ReLU mask flips near zero, ~2% at l1 = 1e-4)
            mu = ref.optim_states.mu if hasattr(ref.optim_states, "mu") else ref.optim_states[0].mu
            for k in fused.m:
                if k not in mu:
                    continue
                for g in range(G):
                    a, b = fused.m[k][g].float(), mu[k][g].float().reshape(fused.m[k][g].shape)
                    e = float((a - b).norm() / b.norm().clamp_min(1e-30))
                    assert e <= 5e-2, (k, g, e)
    for k, v in fused.params.items():
        init = torch.stack([m[0][k] for m in models]).to(DEV)
        mv_f, mv_r = (v - init).flatten(), (ref.params[k] - init).flatten()
        # Adam turns tiny gradients into +-lr steps, so compare the update direction, not max error
        cos = torch.nn.functional.cosine_similarity(mv_f, mv_r, dim=0).item()
        rel = ((mv_f - mv_r).abs().mean() / mv_r.abs().mean()).item()
        assert cos > 0.97 and rel < 0.2, (k, cos, rel)


def test_graph_replay_matches_eager():
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.models.signatures import FunctionalSAE

    torch.manual_seed(4)
    d, n, B = 256, 512, 256
    models = [FunctionalSAE.init(d, n, l1, device=DEV) for l1 in (1e-4, 1e-3)]
    eager = FusedSAEEnsemble(models, FunctionalSAE, batch_size=B, device=DEV)
    graph = FusedSAEEnsemble(models, FunctionalSAE, batch_size=B, device=DEV).enable_graph()
    xs = [torch.randn(B, d, device=DEV).to(torch.bfloat16) for _ in range(4)]
    for x in xs:
        eager.step_batch(x)
        graph.step_batch(x)
    torch.cuda.synchronize()
    assert int(graph.step_dev.item()) == 4 and graph.step_count == 4
    for k in eager.params:
        torch.testing.assert_close(graph.params[k], eager.params[k], rtol=0, atol=0)
    torch.testing.assert_close(graph.out, eager.out, rtol=0, atol=0)


# block-per-row, wave-per-row, block (PL=48), block-radix (n % 4 != 0), block (PL=64)
@pytest.mark.parametrize("n", [6144, 1000, 12288, 1002, 16000])
def test_topk_select_exact(n):
    from sparse_coding__amd.ops import topk as T

    torch.manual_seed(6)
    G, B = 3, 64
    scores = torch.randn(G, B, n, device=DEV)
    scores[0, 0, :10] = 5.0  # ties at the threshold
    scores[1, 2, :] = 0.0  # every key tied: the bracket overflows and the full bisection runs
    scores[2, 1, 100:400] = 0.75  # a crowded bucket: 300 equal keys straddle the threshold
    scores[2, 1, 400:] = -1.0
    k = torch.tensor([1, 32, 150], device=DEV, dtype=torch.int32)
    idx, val = T.topk_select(scores, k, 150, relu=False)
    for g in range(G):
        kg = int(k[g])
        ref = torch.topk(scores[g], kg, dim=-1).values.sort(dim=-1).values
        got = val[g, :, :kg].sort(dim=-1).values
        torch.testing.assert_close(got, ref)
        torch.testing.assert_close(scores[g].gather(-1, idx[g, :, :kg].long()), val[g, :, :kg])
        assert (val[g, :, kg:] == 0).all()
        assert idx[g, :, :kg].sort(-1).values.diff(dim=-1).gt(0).all()  # no duplicates
    assert int(idx[0, 0, 0]) == 0  # k=1 among 10 tied maxima: thread-major order takes index 0
    idx2, val2 = T.topk_select(scores, k, 150, relu=False)
    assert torch.equal(idx2, idx) and torch.equal(val2, val)
    ia, va = T.topk_select(scores, k, 150, absolute=True, relu=False)
    ref = torch.topk(scores[2].abs(), 150, dim=-1).values.sort(-1).values
    torch.testing.assert_close(va[2].abs().sort(-1).values, ref)


@pytest.mark.parametrize("n", [6144, 1024])
def test_topk_select_bf16_picks_are_fp32_topk(n):
    """Select on the scores GEMM's bf16 output: the picks are the top-k of the fp32 scores the GEMM
    accumulated (bf16 ties at the threshold ranked by exact recomputes from x and D), the values
    are the bf16 scores; clustered near-equal scores, duplicated atoms and an all-zero row (heavy
    ties: full-bisection fallback, column order)."""
    from sparse_coding__amd.ops import gemm as gemm_ops
    from sparse_coding__amd.ops import topk as T

    torch.manual_seed(9)
    G, B, d = 3, 128, 768
    D = torch.nn.functional.normalize(torch.randn(G, n, d, device=DEV), dim=-1)
    # model 0: 40 atoms within bf16 resolution of atom 100 -> their scores cluster on rows aligned with it
    D[0, 100:140] = D[0, 100] + 2e-3 * torch.randn(40, d, device=DEV)
    D[1, 7] = D[1, 5]  # a duplicated atom: exactly equal scores, the lower column first
    D = D.to(torch.bfloat16).contiguous()
    x = torch.randn(B, d, device=DEV)
    x[:32] += 10.0 * D[0, 100].float()
    x[40] = 0.0  # every score zero
    x = x.to(torch.bfloat16).contiguous()
    sb = torch.empty(G, B, n, device=DEV, dtype=torch.bfloat16)
    gemm_ops.matmul_nt(x, D, sb)
    exact = torch.einsum("bd,gnd->gbn", x.double(), D.double())
    k = torch.tensor([8, 64, 128], device=DEV, dtype=torch.int32)
    idx, val = T.topk_select(sb, k, 128, x=x, D=D)
    torch.cuda.synchronize()
    tol = 1e-5 * exact.abs().amax().item()
    nres = 0
    for g in range(G):
        kg = int(k[g])
        pick = idx[g, :, :kg].long()
        assert pick.sort(-1).values.diff(dim=-1).gt(0).all()  # no duplicates
        assert (idx[g, :, kg:] == 0).all() and (val[g, :, kg:] == 0).all()
        assert torch.equal(val[g, :, :kg], sb[g].gather(-1, pick).float().clamp(min=0))
        e = exact[g]
        kth = e.topk(kg, dim=-1).values[:, -1:]
        got = e.gather(-1, pick)
        mask = torch.ones_like(e, dtype=torch.bool).scatter_(-1, pick, False)
        rows = torch.arange(B, device=DEV) != 40
        assert (got[rows] >= kth[rows] - tol).all()  # every pick is in the fp32 top-k ...
        assert (e[rows].masked_fill(~mask[rows], -1e30) <= kth[rows] + tol).all()  # ... and nothing above it left out
        # rows whose bf16 threshold key has more ties than slots left: the exact path ranked them
        sf = sb[g].float()
        kb = sf.topk(kg, dim=-1).values[:, -1:]
        nres += int(((sf == kb).sum(-1) > kg - (sf > kb).sum(-1))[rows].sum())
    assert nres > 0  # the clustered rows exercise the exact tie resolution
    assert set(idx[0, 40, :8].tolist()) == set(range(8))  # all-zero row: ties by column
    has5, has7 = (idx[1, :, :64] == 5).any(-1), (idx[1, :, :64] == 7).any(-1)
    assert not (has7 & ~has5).any()  # equal exact scores: the lower column first
    idx2, val2 = T.topk_select(sb, k, 128, x=x, D=D)
    assert torch.equal(idx2, idx) and torch.equal(val2, val)  # deterministic


def test_topk_select_bf16_fallback_paths_are_a_bf16_topk():
    """The bf16 select past its exact-tie limits (ops/topk.py docstring): k > 256 (no bracket path) and
    more than TIE_CAP = 64 keys tied at the k-th bf16 key.  There the picks are still a top-k of the
    bf16 keys -- every pick >= the k-th largest bf16 score, nothing above it left out, no duplicates --
    with ties at the threshold taken in column order (the lowest tied columns)."""
    from sparse_coding__amd.ops import topk as T

    torch.manual_seed(17)
    G, B, n = 2, 64, 2048
    scores = torch.randn(G, B, n, device=DEV)
    # model 1: 200 columns share one value just below the top 100 -> > 64 ties at the threshold
    scores[1, :, 500:700] = -5.0
    scores[1, :, 1000:1100] = 10.0 + torch.rand(B, 100, device=DEV)
    scores[1, :, :500] = -9.0
    scores[1, :, 700:1000] = -9.0
    scores[1, :, 1100:] = -9.0
    sb = scores.to(torch.bfloat16)
    k = torch.tensor([300, 150], device=DEV, dtype=torch.int32)  # k > 256; 100 + 50 of 200 tied
    idx, val = T.topk_select(sb, k, 300)
    torch.cuda.synchronize()
    sf = sb.float()
    for g in range(G):
        kg = int(k[g])
        pick = idx[g, :, :kg].long()
        assert pick.sort(-1).values.diff(dim=-1).gt(0).all()  # no duplicates
        kth = sf[g].topk(kg, dim=-1).values[:, -1:]
        assert (sf[g].gather(-1, pick) >= kth).all()
        rest = sf[g].scatter(-1, pick, float("-inf"))
        assert (rest <= kth).all()
        assert torch.equal(val[g, :, :kg], sf[g].gather(-1, pick).clamp(min=0))
    tied = idx[1, :, :150].long()
    chosen = tied[(tied >= 500) & (tied < 700)].view(B, -1)  # the 50 tied columns taken per row
    assert chosen.shape[1] == 50 and torch.equal(chosen.sort(-1).values,
                                                 torch.arange(500, 550, device=DEV).expand(B, 50))


def test_topk_scatter_and_clear_roundtrip():
    from sparse_coding__amd.ops import topk as T

    torch.manual_seed(4)
    G, B, n = 3, 128, 512
    scores = torch.randn(G, B, n, device=DEV)
    k = torch.tensor([1, 7, 40], dtype=torch.int32, device=DEV)
    idx, val = T.topk_select(scores, k, 40)
    code = torch.zeros(G, B, n, device=DEV, dtype=torch.bfloat16)
    T.scatter(idx, val, k, code)
    ref = torch.zeros(G, B, n, device=DEV).scatter_add_(-1, idx.long(), val)
    torch.testing.assert_close(code.float(), ref.to(torch.bfloat16).float(), rtol=0, atol=0)
    other = torch.zeros_like(code)
    T.clear(idx, code, other)
    assert int(code.ne(0).sum()) == 0


@pytest.mark.parametrize("sparse_k,grad_dtype", [(0, "fp32"), (0, "bf16"), (1000, "fp32"), ("auto", "bf16"),
                                                (8, "bf16")])
def test_fused_topk_matches_autograd(sparse_k, grad_dtype):
    from sparse_coding__amd.engine.topk import FusedTopKEnsemble
    from sparse_coding__amd.models.topk import TopKEncoder

    torch.manual_seed(7)
    d, n, B = 256, 1024, 256
    models = [TopKEncoder.init(d, n, k, device=DEV) for k in (4, 16, 64)]
    eng = FusedTopKEnsemble(models, batch_size=B, device=DEV, lr=1e-3, sparse_k=sparse_k, grad_dtype=grad_dtype)
    assert eng.g.dtype == (torch.bfloat16 if grad_dtype == "bf16" else torch.float32)
    assert eng.sparse_g == {0: 0, 1000: 3}.get(sparse_k, eng.sparse_g)
    x = torch.randn(B, d, device=DEV).to(torch.bfloat16)
    mse = eng.step_batch(x)
    torch.cuda.synchronize()
    for i, (p, b) in enumerate(models):
        pr = {"dict": p["dict"].clone().requires_grad_()}
        loss, _ = TopKEncoder.loss(pr, b, x.float())
        torch.testing.assert_close(mse[i], loss.detach(), rtol=2e-2, atol=1e-4)
        loss.backward()
        g_ref = pr["dict"].grad
        # one Adam step from zero moments moves every parameter by ~lr * sign(g)
        moved = eng.params["dict"][i] - p["dict"]
        agree = (torch.sign(moved) == -torch.sign(g_ref)) | (g_ref.abs() < 1e-7)
        assert agree.float().mean() > 0.97, agree.float().mean()


@pytest.mark.parametrize("grad_dtype", ["fp32", "bf16"])
def test_fused_topk_gradient_config4_matches_fp32_autograd(grad_dtype):
    """Config 4 shape (GPT-2-small residual d = 768, n = 6144, B = 2048, k = 8 .. 128): the
    dictionary gradient of EVERY model -- slot-list path for the small k, dense GEMM for the
    rest -- against fp32 autograd of the top-k loss at the engine's own picks and the bf16 operands it
    multiplies; relative Frobenius error <= 1e-2."""
    from sparse_coding__amd.engine.topk import FusedTopKEnsemble
    from sparse_coding__amd.models.topk import TopKEncoder

    torch.manual_seed(18)
    d, n, B = 768, 6144, 2048
    ks = [8, 16, 24, 32, 48, 64, 96, 128]
    models = [TopKEncoder.init(d, n, k, device=DEV) for k in ks]
    eng = FusedTopKEnsemble(models, batch_size=B, device=DEV, lr=1e-3, grad_dtype=grad_dtype)
    assert 0 < eng.sparse_g < len(ks)  # both wgrad paths are exercised
    D0 = eng.shadow.float().clone()
    feats = torch.nn.functional.normalize(torch.randn(4096, d, device=DEV), dim=-1)
    x = ((torch.relu(torch.randn(B, 4096, device=DEV) - 1.5) * 3.0) @ feats).to(torch.bfloat16)
    mse = eng.step_batch(x)
    torch.cuda.synchronize()
    xf = x.float()
    for g, k in enumerate(ks):
        Dl = D0[g].clone().requires_grad_()
        sel = eng.idx[g, :, :k].long()
        Ds = Dl[sel]  # [B, k, d]
        c = torch.relu(torch.einsum("bd,bkd->bk", xf, Ds))
        loss = (torch.einsum("bk,bkd->bd", c, Ds) - xf).pow(2).mean()
        loss.backward()
        ref = Dl.grad
        rel = ((eng.g[g].float() - ref).norm() / ref.norm()).item()
        assert rel < 1e-2, (g, k, g < eng.sparse_g, rel)
        torch.testing.assert_close(mse[g], loss.detach(), rtol=1e-2, atol=1e-5)


def test_topk_tail_matches_separate_launches():
    """The fused top-k tail (one launch: row Adam + per-model MSE + step counter) == the separate
    Adam launch, torch reductions and counter increment: masters, moments, shadows bit-equal over
    three steps, MSE to fp32 rounding, the device counter advanced once per step."""
    from sparse_coding__amd.engine.topk import FusedTopKEnsemble
    from sparse_coding__amd.models.topk import TopKEncoder

    torch.manual_seed(23)
    d, n, B = 768, 1024, 256
    models = [TopKEncoder.init(d, n, k, device=DEV) for k in (4, 16, 64)]
    fused, split = (FusedTopKEnsemble(models, batch_size=B, device=DEV, lr=1e-3) for _ in range(2))
    assert fused._tail
    split._tail = False
    for t in range(3):
        x = torch.randn(B, d, device=DEV).to(torch.bfloat16)
        mf, ms = fused.step_batch(x).clone(), split.step_batch(x).clone()
        torch.cuda.synchronize()
        torch.testing.assert_close(mf, ms, rtol=1e-5, atol=0)
        assert int(fused.step_dev.item()) == int(split.step_dev.item()) == t + 1
    for a, b in ((fused.params["dict"], split.params["dict"]), (fused.m["dict"], split.m["dict"]),
                 (fused.v["dict"], split.v["dict"]), (fused.shadow, split.shadow), (fused.norms, split.norms)):
        assert torch.equal(a, b)
    assert not fused._ticket.any()  # the completion counters reset themselves


def test_fused_topk_graph_matches_eager():
    """The two captured step graphs (alternating pick buffers: step t clears step t-1's picks
    in the dense buffers) == eager steps, bitwise, over several steps."""
    from sparse_coding__amd.engine.topk import FusedTopKEnsemble
    from sparse_coding__amd.models.topk import TopKEncoder

    torch.manual_seed(13)
    d, n, B = 256, 1024, 256
    models = [TopKEncoder.init(d, n, k, device=DEV) for k in (4, 16, 64)]
    engs = [FusedTopKEnsemble(models, batch_size=B, device=DEV, lr=1e-3, sparse_k=8) for _ in range(2)]
    engs[1].enable_graph()
    assert engs[0].sparse_g == 1
    for s in range(5):
        x = torch.randn(B, d, device=DEV).to(torch.bfloat16)
        mse = [e.step_batch(x).clone() for e in engs]
        torch.cuda.synchronize()
        assert torch.equal(mse[0], mse[1]), s
        assert torch.equal(engs[0].g, engs[1].g), s
        assert torch.equal(engs[0].idx, engs[1].idx), s
    assert torch.equal(engs[0].params["dict"], engs[1].params["dict"])
    assert int(engs[1].step_dev) == 5
    # the dense buffers hold exactly the last step's picks (older ones were cleared)
    e = engs[1]
    for g in range(3):
        nz = e.codebuf[g].ne(0).sum().item()
        assert nz <= B * int(e.k[g]), (g, nz)


def test_gather_rows_matches_index_select():
    from sparse_coding__amd.data.ring import DeviceRing
    from sparse_coding__amd.ops.rows import gather_rows

    torch.manual_seed(9)
    buf = torch.randn(5000, 512, device=DEV).to(torch.bfloat16)
    idx = torch.randint(0, 5000, (2048,), device=DEV)
    out = torch.empty(2048, 512, device=DEV, dtype=torch.bfloat16)
    gather_rows(buf, idx, out=out)
    assert torch.equal(out, buf.index_select(0, idx))
    assert torch.equal(gather_rows(buf[:, :8].contiguous(), idx[:3]), buf[idx[:3], :8])
    ring = DeviceRing(4096, 512, device=DEV)
    ring.push(buf[:4096])
    rows, ridx = ring.sample_shard(1024, 1, 2, return_index=True)
    assert torch.equal(rows, ring.view().index_select(0, ridx))


@pytest.mark.parametrize("form", ["direct", "gram", "direct_rt2"])
@pytest.mark.parametrize("G,B,n,d", [(2, 64, 512, 512), (3, 32, 2048, 512), (1, 48, 1024, 1024), (2, 256, 512, 1024),
                                     (2, 64, 256, 256), (2, 64, 512, 256)])
def test_fista_kernel_matches_oracle(G, B, n, d, form):
    from sparse_coding__amd.ops import fista as F

    if form == "gram" and n not in F.GRAM_N:
        pytest.skip("gram form instantiated for n <= 1024")
    rows = 0
    if form == "direct_rt2":  # the 32-row workgroups (instantiated for n/128 <= 4, d/128 in 2, 4, 8)
        if B % 32 or (d // 128, n // 128) not in {(2, 2), (2, 4), (4, 4), (8, 4)}:
            pytest.skip("no 32-row variant for this shape")
        rows, form = 32, "direct"

    torch.manual_seed(8)
    D = torch.nn.functional.normalize(torch.randn(G, n, d, device=DEV), dim=-1)
    X = torch.randn(B, d, device=DEV)
    A0 = torch.relu(torch.randn(G, B, n, device=DEV)) * 0.05
    lam = torch.linspace(1e-3, 3e-2, G, device=DEV)
    eta = F.step_size(D)
    # oracle on the same bf16-rounded operands the kernel multiplies
    Db = D.to(torch.bfloat16).float()
    Xb = X.to(torch.bfloat16).float()
    A_ref, _ = F.fista_torch(Xb, Db, lam, A0, iters=30, eta=eta)
    R_ref = X - torch.bmm(A_ref, D)
    A, R = F.fista(X, D, lam, A0, iters=30, eta=eta, backend="hip", form=form, rows=rows)
    torch.cuda.synchronize()
    err_a = (A - A_ref).abs().max().item() / (A_ref.abs().max().item() + 1e-6)
    err_r = (R - R_ref).abs().max().item() / (R_ref.abs().max().item() + 1e-6)
    assert err_a < 3e-2 and err_r < 3e-2, (err_a, err_r)
    def obj(A_, R_):
        return 0.5 * R_.pow(2).sum((1, 2)) + lam * A_.abs().sum((1, 2))
    torch.testing.assert_close(obj(A, R), obj(A_ref, R_ref), rtol=1e-2, atol=1e-3)


def test_fused_and_topk_steps_deterministic_under_debug_mode():
    """Every training-path kernel is deterministic (no float atomics): two runs from the
    same state agree bitwise; debug mode also syncs after each launch."""
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.engine.topk import FusedTopKEnsemble
    from sparse_coding__amd.models.signatures import FunctionalSAE
    from sparse_coding__amd.models.topk import TopKEncoder
    from sparse_coding__amd.utils import debug

    xs = [torch.randn(256, 256, device=DEV).to(torch.bfloat16) for _ in range(3)]

    def make_sae():
        torch.manual_seed(9)
        return FusedSAEEnsemble([FunctionalSAE.init(256, 512, l1, device=DEV) for l1 in (1e-4, 1e-3)],
                                FunctionalSAE, batch_size=256, device=DEV)

    def run_sae(e):
        for x in xs:
            e.step_batch(x)
        return {**e.params, "out": e.out}

    def make_topk():
        torch.manual_seed(9)
        return FusedTopKEnsemble([TopKEncoder.init(256, 512, k, device=DEV) for k in (4, 16)], batch_size=256,
                                 device=DEV)

    def run_topk(e):
        for x in xs:
            e.step_batch(x)
        return dict(e.params)

    with debug.debug_mode():
        debug.assert_deterministic(make_sae, run_sae)
        debug.assert_deterministic(make_topk, run_topk)


def test_fused_tied_with_affine_centering_matches_closed_form():
    """Non-identity centering buffers run in the fused engine (x R^T GEMM + elementwise)."""
    from sparse_coding__amd.engine.analytic import AnalyticSAEEnsemble
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.models.signatures import FunctionalTiedSAE

    torch.manual_seed(11)
    d, n, B = 256, 512, 256
    models = []
    for l1 in (1e-4, 1e-3):
        rot = torch.linalg.qr(torch.randn(d, d))[0]
        models.append(FunctionalTiedSAE.init(d, n, l1, rotation=rot, translation=0.1 * torch.randn(d),
                                             scaling=torch.rand(d) + 0.5))
    dev_models = [({k: v.to(DEV) for k, v in p.items()}, {k: v.to(DEV) for k, v in b.items()}) for p, b in models]
    fused = FusedSAEEnsemble(dev_models, FunctionalTiedSAE, batch_size=B, device=DEV)
    ref = AnalyticSAEEnsemble(dev_models, FunctionalTiedSAE, device=DEV)
    for _ in range(4):
        x = torch.randn(B, d, device=DEV).to(torch.bfloat16)
        out = fused.step_batch(x)
        losses, _ = ref.step_batch(x.float())
        torch.testing.assert_close(out[:, 1], losses["l_reconstruction"], rtol=3e-2, atol=1e-4)
    init = torch.stack([m[0]["encoder"] for m in dev_models])
    du, dr = (fused.params["encoder"] - init).flatten(), (ref.params["encoder"] - init).flatten()
    assert torch.nn.functional.cosine_similarity(du, dr, dim=0).item() > 0.97


def test_fused_evaluate_matches_metrics():
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.eval.metrics import batched_fvu_l0
    from sparse_coding__amd.models.signatures import FunctionalSAE

    torch.manual_seed(12)
    d, n, B = 256, 512, 256
    models = [FunctionalSAE.init(d, n, l1, device=DEV) for l1 in (1e-4, 1e-2)]
    e = FusedSAEEnsemble(models, FunctionalSAE, batch_size=B, device=DEV)
    feats = torch.nn.functional.normalize(torch.randn(1024, d, device=DEV), dim=-1)
    for _ in range(20):
        e.step_batch((torch.relu(torch.randn(B, 1024, device=DEV) - 2) @ feats).to(torch.bfloat16))
    rows = (torch.relu(torch.randn(4 * B, 1024, device=DEV) - 2) @ feats).to(torch.bfloat16)
    fvu, l0 = e.evaluate(rows)
    for g, ld in enumerate(e.to_learned_dicts(DEV)):
        f_ref, l_ref = batched_fvu_l0(ld, rows.float())
        assert abs(float(fvu[g]) - f_ref) < 0.02 + 0.02 * f_ref, (g, float(fvu[g]), f_ref)
        assert abs(float(l0[g]) - l_ref) < 0.05 * max(l_ref, 1.0), (g, float(l0[g]), l_ref)


@pytest.mark.parametrize("ksplit", [2, 4])
@pytest.mark.parametrize("nseg", [1, 2])
def test_weight_grads_split_k(ksplit, nseg):
    """Split-K weight gradients: the partial slabs sum to the fp32 reference product."""
    from sparse_coding__amd.ops import gemm

    torch.manual_seed(11)
    G, Bk, n, d = 2, 1024, 512, 256
    pairs, ref = [], torch.zeros(G, n, d, device=DEV)
    for _ in range(nseg):
        A, Bm = _bf(G, Bk, n), _bf(G, Bk, d)
        pairs.append((A, Bm))
        ref += A.float().transpose(1, 2) @ Bm.float()
    out = torch.empty(ksplit, G, n, d, device=DEV)
    gemm.weight_grads([pairs], [out], 0.5, ksplit=ksplit)
    _close(out.sum(0), 0.5 * ref, rtol=1e-3, atol=1e-3)
    # each slab is a genuine partial (not the full product written ksplit times)
    assert (out[0] - 0.5 * ref).abs().max() > 1.0


def test_fused_step_wgrad_split_matches_unsplit():
    """The engine's split-K weight gradients (summed by the Adam kernel) give the same
    trajectory as the single-slab path."""
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.models.signatures import FunctionalSAE

    torch.manual_seed(12)
    d, n, B = 256, 512, 2048
    models = [FunctionalSAE.init(d, n, l1, device=DEV) for l1 in (1e-4, 1e-3)]
    a = FusedSAEEnsemble(models, FunctionalSAE, batch_size=B, device=DEV, wgrad_split=1)
    b = FusedSAEEnsemble(models, FunctionalSAE, batch_size=B, device=DEV, wgrad_split=4)
    assert b.g_parts is not None and a.g_parts is None
    for _ in range(3):
        x = torch.randn(B, d, device=DEV).to(torch.bfloat16)
        a.step_batch(x)
        b.step_batch(x)
    torch.cuda.synchronize()
    for k in a.params:
        init = torch.stack([m[0][k] for m in models]).to(DEV)
        ua, ub = (a.params[k] - init).flatten(), (b.params[k] - init).flatten()
        # fp32 summation order differs between slabs; Adam maps near-zero gradients to
        # O(lr) steps, so compare the updates' direction and mean deviation
        cos = torch.nn.functional.cosine_similarity(ua, ub, dim=0).item()
        rel = ((ua - ub).abs().mean() / ua.abs().mean()).item()
        assert cos > 0.999 and rel < 1e-2, (k, cos, rel)
    torch.testing.assert_close(b.out, a.out, rtol=1e-3, atol=1e-5)


def test_graph_static_inputs_match_eager():
    """Graphs captured on two registered input buffers (double-buffered batches) replay
    the same step as eager launches on those buffers."""
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.models.signatures import FunctionalSAE

    torch.manual_seed(13)
    d, n, B = 256, 512, 256
    models = [FunctionalSAE.init(d, n, l1, device=DEV) for l1 in (1e-4, 1e-3)]
    eager = FusedSAEEnsemble(models, FunctionalSAE, batch_size=B, device=DEV)
    graph = FusedSAEEnsemble(models, FunctionalSAE, batch_size=B, device=DEV).enable_graph()
    bufs = [torch.empty(B, d, device=DEV, dtype=torch.bfloat16) for _ in range(2)]
    for t in bufs:
        graph.add_static_input(t)
    for i in range(4):
        x = torch.randn(B, d, device=DEV).to(torch.bfloat16)
        bufs[i % 2].copy_(x)
        eager.step_batch(x)
        graph.step_batch(bufs[i % 2])
    torch.cuda.synchronize()
    for k in eager.params:
        torch.testing.assert_close(graph.params[k], eager.params[k], rtol=0, atol=0)


@pytest.mark.parametrize("n", [512, 1024])
def test_fista_gram_row_tiles_match(n):
    """The 32-row Gram solver (two row tiles, column passes, double-buffered LDS) is
    bit-identical to the 16-row one, which test_fista_kernel_matches_oracle pins."""
    from sparse_coding__amd.ops import fista as F

    torch.manual_seed(9)
    G, B = 4, 4096  # G * B / 32 >= 512 workgroups selects the 32-row kernel
    D = torch.nn.functional.normalize(torch.randn(G, n, n, device=DEV), dim=-1)
    X = torch.randn(B, n, device=DEV) * 0.3
    A0 = torch.relu(torch.randn(G, B, n, device=DEV)) * 0.02
    lam = torch.linspace(1e-3, 1e-2, G, device=DEV)
    eta = F.step_size(D)
    A2, _ = F.fista(X, D, lam, A0, iters=12, eta=eta, backend="hip", with_res=False, form="gram")
    A1, _ = F.fista(X, D, lam, A0, iters=12, eta=eta, backend="hip", with_res=False, form="gram", rows=16)
    torch.cuda.synchronize()
    assert torch.equal(A1, A2)
    assert A1.abs().sum() > 0


@pytest.mark.parametrize("kind", ["reverse", "threshold", "tied_centered"])
def test_fused_activation_variants_match_functional_ensemble(kind):
    """Reverse (K10), smooth-threshold (K11) and learned-centering tied (C8) SAEs on the
    fused engine vs the eager autograd ensemble: losses per step and the direction of
    every parameter's update."""
    from sparse_coding__amd.engine.ensemble import FunctionalEnsemble
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.engine.optim import adam
    from sparse_coding__amd.models.signatures import (FunctionalReverseSAE, FunctionalThresholdingSAE,
                                                      FunctionalTiedCenteredSAE)

    torch.manual_seed(5)
    sig = {"reverse": FunctionalReverseSAE, "threshold": FunctionalThresholdingSAE,
           "tied_centered": FunctionalTiedCenteredSAE}[kind]
    d, n, B = 256, 512, 256
    models = [sig.init(d, n, l1, device=DEV) for l1 in (1e-4, 1e-3, 1e-2)]
    for p, _ in models:
        if kind == "reverse":
            p["encoder_bias"].uniform_(-0.2, 0.2)
        elif kind == "tied_centered":
            # sparse codes: with ~half the 512 atoms active their span covers all of d = 256
            # and the two terms of the center gradient cancel to bf16 noise
            p["encoder_bias"].uniform_(-1.2, -0.8)
            p["center"].normal_(0.0, 0.3)
        else:
            p["activation_scale"].uniform_(0.7, 1.3)
            p["activation_gain"].uniform_(-0.2, 0.4)
            p["centering"].normal_(0.0, 0.05)
    ref = FunctionalEnsemble([({k: v.clone() for k, v in p.items()}, b) for p, b in models], sig, adam,
                             {"lr": 1e-3}, device=DEV)
    fused = FusedSAEEnsemble(models, sig, lr=1e-3, batch_size=B, device=DEV)
    assert fused.kind == ("tied" if kind == "tied_centered" else kind)
    assert fused.learned_center == (kind == "tied_centered")
    feats = torch.nn.functional.normalize(torch.randn(1024, d, device=DEV), dim=-1)
    for step in range(5):
        codes = torch.relu(torch.randn(B, 1024, device=DEV) - 1.5) * 3.0
        x = (codes @ feats).to(torch.bfloat16)
        loss_ref, _ = ref.step_batch(x.float())
        out = fused.step_batch(x)
        torch.cuda.synchronize()
        torch.testing.assert_close(out[:, 1], loss_ref["l_reconstruction"], rtol=3e-2, atol=1e-4)
        torch.testing.assert_close(out[:, 2], loss_ref["l_l1"], rtol=5e-2, atol=1e-5)
        assert float(out[:, 4].min()) > 0.5, "codes must be active for the test to mean anything"
    for k, v in fused.params.items():
        init = torch.stack([m[0][k] for m in models]).to(DEV)
        mv_f, mv_r = (v - init).flatten(), (ref.params[k] - init).flatten()
        if mv_r.abs().max() == 0:  # reverse SAE bias: no gradient through the codes, no decay
            assert mv_f.abs().max() == 0, k
            continue
        cos = torch.nn.functional.cosine_similarity(mv_f, mv_r, dim=0).item()
        rel = ((mv_f - mv_r).abs().mean() / mv_r.abs().mean()).item()
        print(kind, k, "cos", round(cos, 4), "rel", round(rel, 4))
        assert cos > 0.95 and rel < 0.25, (k, cos, rel)
    # evaluate() uses the same epilogues
    fvu, l0 = fused.evaluate(x)
    for g, ld in enumerate(fused.to_learned_dicts(DEV)):
        xf = x.float()
        x_hat = ld.predict(xf)
        f_ref = float((x_hat - xf).pow(2).sum() / (xf - xf.mean(0)).pow(2).sum())
        assert abs(float(fvu[g]) - f_ref) < 0.02 + 0.03 * f_ref, (g, float(fvu[g]), f_ref)


@pytest.mark.parametrize("G,M,N,K", [(1, 128, 128, 64), (3, 300, 517, 200), (2, 1024, 256, 512)])
def test_rowmax_nt_matches_torch(G, M, N, K):
    """EPI_ROWMAX (max cosine similarity, K20) against a torch fp32 max over A B^T."""
    from sparse_coding__amd.ops import gemm

    a = torch.nn.functional.normalize(torch.randn(G, M, K, device=DEV), dim=-1).to(torch.bfloat16)
    b = torch.nn.functional.normalize(torch.randn(G, N, K, device=DEV), dim=-1).to(torch.bfloat16)
    ref = torch.bmm(a.float(), b.float().transpose(1, 2)).amax(-1)
    got = gemm.rowmax_nt(a, b)
    assert got.shape == (G, M)
    torch.testing.assert_close(got, ref, rtol=1e-3, atol=1e-3)
    got2 = gemm.rowmax_nt(a[0], b[0], alpha=-1.0)  # 2-D form; alpha flips to a row min
    torch.testing.assert_close(got2, -torch.mm(a[0].float(), b[0].float().T).amin(-1), rtol=1e-3, atol=1e-3)


def test_mmcs_fused_path_matches_fp32():
    from sparse_coding__amd.eval import metrics
    from sparse_coding__amd.models.learned_dict import UntiedSAE

    torch.manual_seed(2)
    d = 512
    lds = [UntiedSAE(torch.randn(4096, d, device=DEV), torch.randn(4096, d, device=DEV),
                     torch.zeros(4096, device=DEV)) for _ in range(2)]
    exact = metrics.max_cosine(lds[0].get_learned_dict(), lds[1].get_learned_dict(), fused=False)
    fused = metrics.max_cosine(lds[0].get_learned_dict(), lds[1].get_learned_dict(), fused=True)
    torch.testing.assert_close(fused, exact, rtol=0, atol=6e-3)
    assert abs(float(metrics.mmcs(lds[0], lds[1])) - float(exact.mean())) < 2e-3


@pytest.mark.parametrize("M,N,K", [(300, 517, 200), (4096, 4100, 512)])
def test_rowmax_nt_256_blocks(M, N, K):
    """The 256x256-block EPI_ROWMAX path (padding to 256; auto-selected from 16M entries)."""
    from sparse_coding__amd.ops import gemm

    torch.manual_seed(3)
    a = torch.nn.functional.normalize(torch.randn(M, K, device=DEV), dim=-1).to(torch.bfloat16)
    b = torch.nn.functional.normalize(torch.randn(N, K, device=DEV), dim=-1).to(torch.bfloat16)
    ref = torch.mm(a.float(), b.float().T).amax(-1)
    torch.testing.assert_close(gemm.rowmax_nt(a, b, cfg=3), ref, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(gemm.rowmax_nt(a, b), ref, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("normalize", ["column", "row"])
@pytest.mark.parametrize("nonneg", [False, True])
def test_fista_dictionary_update_on_device(normalize, nonneg):
    """Hessian-diagonal EMA and the quadratic basis update (reference autoencoders/fista.py:
    88-96, 131-138) as HIP kernels + the MFMA A^T Res GEMM, against the fp32 torch path."""
    from sparse_coding__amd.ops import fista as F

    torch.manual_seed(12)
    G, B, n, d = 3, 512, 256, 384
    D = torch.nn.functional.normalize(torch.randn(G, n, d, device=DEV), dim=-1)
    A = torch.relu(torch.randn(G, B, n, device=DEV) - 1.0)
    Res = torch.randn(G, B, d, device=DEV) * 0.3
    H0 = torch.rand(G, n, device=DEV) * 0.1
    H_ref = F.hessian_ema(H0, A, 300, backend="torch")
    H_hip = F.hessian_ema(H0, A, 300, backend="hip")
    torch.testing.assert_close(H_hip, H_ref, rtol=1e-5, atol=1e-7)
    shadow = torch.empty(G, n, d, device=DEV, dtype=torch.bfloat16)
    ref = F.quadratic_basis_update(D, Res, A, H_ref, 0.001, 0.05, nonneg, normalize, backend="torch")
    got = F.quadratic_basis_update(D, Res, A, H_hip, 0.001, 0.05, nonneg, normalize, backend="hip", shadow_out=shadow)
    torch.cuda.synchronize()
    # the update itself (step 0.05, bf16 GEMM operands) is reproduced to bf16 accuracy
    du_ref, du_got = ref - D, got - D
    rel = float((du_got - du_ref).norm() / du_ref.norm())
    assert rel < 1e-2, rel
    torch.testing.assert_close(shadow.float(), got, rtol=1e-2, atol=1e-2)


def test_fista_gram_hot_path_matches_fp32_dictionary_step():
    """The GPU dictionary step's hot path (``ops.fista.gram_solve``: X D^T / D D^T on the MFMA GEMM, eta
    from the solver's own Gram, the residual from the decoder GEMM's EPI_DEC epilogue in bf16, negated)
    feeding ``quadratic_basis_update(A_bf16=, res_neg_bf16=)`` == the fp32 path (``fista()`` with its
    fp32 residual, fp32 eigenvalue step size, fp32 basis update), to bf16 accuracy; the tracker's eta
    from the Gram bounds the same spectrum as the exact eigh of D D^T."""
    from sparse_coding__amd.models.fista import FistaDictUpdater
    from sparse_coding__amd.ops import fista as F

    torch.manual_seed(21)
    G, B, n, d = 3, 256, 256, 384
    D = torch.nn.functional.normalize(torch.randn(G, n, d, device=DEV), dim=-1)
    X = (torch.randn(B, d, device=DEV) * 0.5).to(torch.bfloat16)
    lam = torch.tensor([1e-3, 1e-2, 5e-2], device=DEV)
    A0 = torch.relu(torch.randn(G, B, n, device=DEV) * 0.1).to(torch.bfloat16)
    assert F.gram_solve_ok(X, D)
    tracker = F.EtaTracker()
    A, Ab, Rn, eta, se = F.gram_solve(X, D, lam, A0, 60, tracker=tracker)
    eta_ref = F.step_size(D, "eigh")
    torch.testing.assert_close(eta, eta_ref, rtol=5e-3, atol=0)  # bf16 Gram vs fp32 spectrum
    assert tracker.space == "ddt" and tracker.v.shape == (G, n, 1)
    A_ref, R_ref = F.fista(X, D, lam, A0, 60, eta, backend="hip", form="gram")
    torch.testing.assert_close(A, A_ref, rtol=0, atol=0)  # the same solver on the same operands
    assert torch.equal(Ab, A.to(torch.bfloat16))
    rel = float((-Rn.float() - R_ref).norm() / R_ref.norm())
    assert rel < 1e-2, rel
    torch.testing.assert_close(se, R_ref.pow(2).sum(dim=(1, 2)), rtol=2e-2, atol=0)
    H = torch.rand(G, n, device=DEV) * 0.1
    ref = F.quadratic_basis_update(D, R_ref, A_ref, H, 0.001, 0.05, backend="torch")
    got = F.quadratic_basis_update(D, None, A, H, 0.001, 0.05, A_bf16=Ab, res_neg_bf16=Rn)
    rel = float(((got - D) - (ref - D)).norm() / (ref - D).norm())
    assert rel < 2e-2, rel
    # the updater takes the hot path on these shapes and matches its fp32 torch form
    hot, ref_u = FistaDictUpdater(num_iter=40), FistaDictUpdater(num_iter=40, backend="torch", eta_method="eigh")
    Dn, res, An = hot(D.clone(), X, A0, lam)
    Dr, res_r, Ar = ref_u(D.clone(), X.float(), A0.float(), lam)
    rel = float(((Dn - D) - (Dr - D)).norm() / (Dr - D).norm())
    assert rel < 5e-2, rel
    assert res.dtype == torch.float32 and res.shape == (G, B, d)


def test_unrolled_fista_hip_adjoint_matches_fp32():
    """FISTA in the loss on the kernels.  Forward: the HIP solver's residual against the fp32
    loop.  Backward: the HIP adjoint sweep (grouped GEMMs + elementwise kernel + the K = T B
    dictionary-gradient GEMM) against the fp32 adjoint (pinned to autograd through the loop in
    tests/test_fista_loss_cpu.py) run over the SAME saved iterate slabs.  (Against the fp32
    trajectory the gradient differs by ~14%: bf16 rounding of D alone flips relu supports along
    the 20 iterations -- measured by CPU emulation, a property of the unrolled objective, not of
    the adjoint.)"""
    from sparse_coding__amd.ops import fista as F

    torch.manual_seed(12)
    G, B, n, d, T = 2, 256, 512, 256, 20
    D = torch.nn.functional.normalize(torch.randn(G, n, d, device=DEV), dim=-1)
    X = torch.randn(B, d, device=DEV)
    c = torch.relu(torch.randn(G, B, n, device=DEV)) * 0.05
    lam = torch.tensor([1e-3, 2e-2], device=DEV)
    eta = F.step_size(D)
    W = torch.randn(G, B, d, device=DEV)
    R_ref = F.unrolled_fista_residual(X, D, lam, c, T, eta, backend="torch")
    mom = F.momentum_schedule(T)
    R, Db, Ys, Rs, As = F.unrolled_forward_hip(X, D, c, lam, eta, T, mom)
    Dh, ch, _ = F.unrolled_backward_hip(W, Db, Ys, Rs, As, eta, mom.tolist(), T)
    Dr, cr, _ = F.unrolled_backward_torch(W, Db.float(), Ys, Rs, As, eta, mom.tolist(), T)
    torch.cuda.synchronize()
    for g in range(G):
        rel = lambda a, b: ((a[g] - b[g]).norm() / b[g].norm()).item()  # noqa: E731
        assert rel(R, R_ref) < 3e-2, rel(R, R_ref)
        assert rel(Dh, Dr) < 1e-2, rel(Dh, Dr)
        assert rel(ch, cr) < 1e-2, rel(ch, cr)
    # the autograd Function routes to exactly these kernels
    D1, c1 = D.clone().requires_grad_(), c.clone().requires_grad_()
    (F.unrolled_fista_residual(X, D1, lam, c1, T, eta, backend="hip") * W).sum().backward()
    torch.testing.assert_close(D1.grad, Dh, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("G,B,n,d", [(2, 256, 512, 512), (4, 4096, 512, 512), (2, 256, 256, 512)])
def test_unrolled_fista_gram_adjoint_matches_fp32(G, B, n, d):
    """Gram-form FISTA in the loss: the slab-saving solve and the reverse sweep in the Gram
    kernel (16- and 32-row workgroups) with the dictionary gradient from M = sum_t Vbar_t^T Y_t
    (no residual slabs) against the fp32 adjoint over the same Y / A slabs (residual slabs
    recomputed in fp32), including d loss / d eta."""
    from sparse_coding__amd.ops import fista as F

    torch.manual_seed(21)
    T = 20
    D = torch.nn.functional.normalize(torch.randn(G, n, d, device=DEV), dim=-1)
    X = torch.randn(B, d, device=DEV)
    c = torch.relu(torch.randn(G, B, n, device=DEV)) * 0.05
    lam = torch.linspace(1e-3, 2e-2, G, device=DEV)
    eta = F.step_size(D)
    W = torch.randn(G, B, d, device=DEV)
    mom = F.momentum_schedule(T)
    R_ref = F.unrolled_fista_residual(X, D, lam, c, T, eta, backend="torch")
    R, st = F.unrolled_forward_gram(X, D, c, lam, eta, T, mom)
    Xb, Db, Gm, Gmf, Ys, As, Qs = st
    C = Xb.float() @ Db.float().transpose(1, 2)  # X D^T per model
    Dg, cg, eg = F.unrolled_backward_gram(W, st, eta, mom.tolist(), T, lam=lam)
    Df = Db.float()
    Rs = (Xb.float() - Ys.float() @ Df.unsqueeze(1)).to(torch.bfloat16)  # Res_t = X - Y_t D per slot
    Dr, cr, er = F.unrolled_backward_torch(W, Df, Ys, Rs, As, eta, mom.tolist(), T, lam=lam)
    torch.cuda.synchronize()
    for g in range(G):
        rel = lambda a, b: ((a[g] - b[g]).norm() / b[g].norm()).item()  # noqa: E731
        assert rel(R, R_ref) < 3e-2, rel(R, R_ref)
        assert rel(Dg, Dr) < 1e-2, rel(Dg, Dr)
        assert rel(cg, cr) < 1e-2, rel(cg, cr)
    # d loss / d eta is a small difference of large terms (~1/10 of them), so it is pinned against
    # an fp32 reverse sweep of the Gram-form iteration the kernels run (same bf16 Gm and Y slab):
    # sum_t <Vbar_t, C - Y_t Gm> - lam sum Vbar_t.  (Against the D-form torch adjoint above the
    # bf16 rounding of Gm alone moves it by several percent: er is reported, not asserted.)
    e_ = eta[:, None, None]
    Gmf = Gm.float()
    Vbar = -(W.float() @ Df.transpose(1, 2)) * (As[:, T - 1] > 0)
    Ynext = torch.zeros_like(Vbar)
    e_ref = torch.zeros(G, device=DEV)
    for t in range(T - 1, -1, -1):
        e_ref += (Vbar * (C - Ys[:, t].float() @ Gmf)).sum((1, 2)) - lam * Vbar.sum((1, 2))
        Yb = Vbar - e_ * (Vbar @ Gmf)
        if t >= 1:
            Vbar = ((1 + mom[t - 1]) * Yb - mom[t] * Ynext) * (As[:, t - 1] > 0)
        Ynext = Yb
    torch.testing.assert_close(eg, e_ref, rtol=1e-2, atol=1e-2 * e_ref.abs().max().item())
    print("etabar kernel", eg.tolist(), "gram fp32", e_ref.tolist(), "D-form fp32", er.tolist())
    # the 16-row adjoint (rows=16) gives the same gradients
    D16, c16, e16 = F.unrolled_backward_gram(W, st, eta, mom.tolist(), T, lam=lam, rows=16)
    torch.testing.assert_close(D16, Dg, rtol=1e-3, atol=1e-3 * Dg.abs().max().item())
    torch.testing.assert_close(e16, eg, rtol=1e-3, atol=1e-3 * eg.abs().max().item())
    # the autograd Function routes to the Gram path for n <= d
    D1, c1 = D.clone().requires_grad_(), c.clone().requires_grad_()
    (F.unrolled_fista_residual(X, D1, lam, c1, T, eta, backend="hip") * W).sum().backward()
    torch.testing.assert_close(D1.grad, Dg, rtol=1e-3, atol=1e-3)


def test_fista_loss_ensemble_trains_on_gpu():
    from sparse_coding__amd.engine.fista_loss import FistaLossEnsemble
    from sparse_coding__amd.models.fista import FunctionalFista

    torch.manual_seed(13)
    d, n, B = 256, 256, 256
    models = [FunctionalFista.init(d, n, l1, device=DEV) for l1 in (1e-4, 1e-3)]
    eng = FistaLossEnsemble(models, lr=1e-3, batch_size=B, device=DEV, num_iter=10, backend="hip")
    x = torch.randn(B, d, device=DEV)
    first = eng.step_batch(x)
    for _ in range(20):
        last = eng.step_batch(x)
    torch.cuda.synchronize()
    assert torch.isfinite(last).all() and (last < first).all(), (first, last)


@pytest.mark.parametrize("T", [1, 5])
def test_fused_fista_loss_gradients_match_autograd(T):
    """FISTA in the loss on the fused engine (tied SAE kernels + Gram solve / adjoint + eta
    term + warm-start gradient through the ReLU) against fp32 autograd of the reference's
    loss2 (FistaLossEnsemble, torch backend) on the same bf16-rounded batch: the raw encoder
    gradient (norm Jacobian applied to the engine's normalised-row gradient), the bias
    gradient and the loss terms."""
    from sparse_coding__amd.engine.fista_loss import FistaLossEnsemble, FusedFistaLossEnsemble
    from sparse_coding__amd.models.fista import FunctionalFista

    torch.manual_seed(22)
    G, d, n, B = 2, 512, 512, 256
    models = [FunctionalFista.init(d, n, l1, device=DEV) for l1 in (1e-3, 1e-2)]
    feats = torch.nn.functional.normalize(torch.randn(1024, d, device=DEV), dim=-1)
    x = ((torch.relu(torch.randn(B, 1024, device=DEV) - 1.0) * 2.0) @ feats).to(torch.bfloat16)
    fused = FusedFistaLossEnsemble(models, lr=1e-3, batch_size=B, device=DEV, num_iter=T)
    ref = FistaLossEnsemble(models, lr=1e-3, batch_size=B, device=DEV, num_iter=T, backend="torch")
    total, parts = ref.losses(x.float())
    total.sum().backward()
    fused.compute_grads(x)
    torch.cuda.synchronize()
    e = fused.engine
    w_hat = e.params["encoder"] / e.norms.unsqueeze(-1)
    gw = e.g_dec
    g_raw = (gw - (gw * w_hat).sum(-1, keepdim=True) * w_hat) / e.norms.unsqueeze(-1)
    g_ref = ref.params["encoder"].grad
    gb, gb_ref = e.g_bias.view(G, n), ref.params["encoder_bias"].grad
    for g in range(G):
        rel_w = ((g_raw[g] - g_ref[g]).norm() / g_ref[g].norm()).item()
        rel_b = ((gb[g] - gb_ref[g]).norm() / gb_ref[g].norm()).item()
        assert rel_w < 3e-2 and rel_b < 3e-2, (g, rel_w, rel_b)
    torch.testing.assert_close(fused.l_fista, parts["l_fista"].detach(), rtol=2e-2, atol=1e-5)
    # a few steps train
    first = fused.step_batch(x).clone()
    for _ in range(10):
        last = fused.step_batch(x)
    torch.cuda.synchronize()
    assert torch.isfinite(last).all() and (last < first).all(), (first, last)


@pytest.mark.parametrize("engine", ["auto", "fused"])
def test_trainer_fista_loss_fused_steps_and_resumes(engine):
    """EnsembleTrainer(objective='fista_loss') on a GPU takes the fused FISTA-in-loss engine (auto
    and explicit), trains, and a checkpoint round trip continues bit-identically."""
    from sparse_coding__amd.engine.trainer import EnsembleTrainer
    from sparse_coding__amd.models.fista import FunctionalFista

    torch.manual_seed(23)
    d, n, B = 512, 512, 256
    models = [FunctionalFista.init(d, n, l1, device=DEV) for l1 in (1e-3, 3e-3)]
    feats = torch.nn.functional.normalize(torch.randn(1024, d, device=DEV), dim=-1)
    xs = [((torch.relu(torch.randn(B, 1024, device=DEV) - 1.0) * 2.0) @ feats).to(torch.bfloat16)
          for _ in range(4)]

    def make():
        return EnsembleTrainer(models, FunctionalFista, lr=1e-3, batch_size=B, device=DEV, engine=engine,
                               objective="fista_loss", fista_loss_iters=5)

    tr = make()
    assert tr.kind == "fista-loss-fused", tr.engine_reason
    first = tr.step(xs[0]).clone()
    for i in range(6):
        last = tr.step(xs[1 + i % 3])
    torch.cuda.synchronize()
    assert torch.isfinite(last).all()
    buf = io.BytesIO()
    torch.save(tr.state_dict(), buf)  # what a checkpoint file holds (copies, not live views)
    buf.seek(0)
    st = torch.load(buf, weights_only=True)
    tr2 = make()
    tr2.load_state_dict(st)
    a = tr.step(xs[0]).clone()
    b = tr2.step(xs[0]).clone()
    torch.cuda.synchronize()
    assert torch.equal(a, b), (a, b)
    assert torch.equal(tr.impl.params["encoder"], tr2.impl.params["encoder"])
    assert torch.equal(tr.impl.params["encoder_bias"], tr2.impl.params["encoder_bias"])
    assert (a <= first).all(), (first, a)


def test_coef_search_hip_matches_torch():
    """Direct coefficient search (reference direct_coef_search.py:52-56) on the persistent
    solver's projected-momentum mode vs the fp32 loop, 3 models at once."""
    from sparse_coding__amd.ops import fista as F

    torch.manual_seed(14)
    G, B, n, d = 3, 64, 512, 256
    D = torch.nn.functional.normalize(torch.randn(G, n, d, device=DEV), dim=-1)
    X = torch.randn(B, d, device=DEV)
    lam = torch.tensor([1e-3, 1e-2, 5e-2], device=DEV)
    lr = torch.tensor([50.0, 50.0, 20.0], device=DEV)
    A = F.coef_search(X, D, lam, lr, 60, backend="hip")
    R = F.coef_search_torch(X, D.to(torch.bfloat16).float(), lam, lr, 60)
    torch.cuda.synchronize()

    def obj(C):
        return ((X - C @ D) ** 2).mean(dim=(1, 2)) + lam * C.abs().sum(-1).mean(-1)

    torch.testing.assert_close(obj(A), obj(R), rtol=1e-2, atol=1e-4)
    # codes: the two lightly regularised models; at lam = 5e-2 (3 % density) the projected
    # momentum iteration is degenerate -- a CPU emulation with bf16 operands lands on codes 64 %
    # away with the same objective to 4 digits
    for g in range(2):
        rel = ((A[g] - R[g]).norm() / R[g].norm()).item()
        assert rel < 3e-2, (g, rel)


def test_fused_topk_encode_matches_reference_encode():
    """FusedTopKEnsemble.encode (padded slots of small-k models must not clobber feature 0)
    against TopKEncoder.encode per model, mixed k."""
    from sparse_coding__amd.engine.topk import FusedTopKEnsemble
    from sparse_coding__amd.models.topk import TopKEncoder

    torch.manual_seed(15)
    d, n, B = 256, 1024, 256
    models = [TopKEncoder.init(d, n, k, device=DEV) for k in (4, 16)]
    eng = FusedTopKEnsemble(models, batch_size=B, device=DEV)
    x = torch.randn(B, d, device=DEV)
    x[:, :] += 10.0 * (eng.shadow[0, 0] + eng.shadow[1, 0]).float()  # feature 0: a real pick of every row
    got = eng.encode(x)
    torch.cuda.synchronize()
    for g, (p, b) in enumerate(models):
        D = eng.shadow[g].float()
        ref = TopKEncoder.encode(x.to(torch.bfloat16).float(), b["sparsity"], D)
        assert bool((got[g, :, 0] > 0).all())
        torch.testing.assert_close(got[g], ref, rtol=1e-3, atol=1e-3)


def test_tied_centered_center_update_direction_at_dense_codes():
    """Learned-centre tied SAE with dense codes (bias 0, about half the atoms on): the two
    terms of the centre gradient largely cancel, so they come from fp32 data (the decoder
    epilogue's fp32 residual column sums, fp32 masters of the PRE-update dictionary).  The
    gradient must match autograd of the eager fp32 ensemble, and one Adam step from zero
    moments (~lr sign(g)) must move the centre the same way."""
    from sparse_coding__amd.engine.ensemble import FunctionalEnsemble
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.engine.optim import adam
    from sparse_coding__amd.models.signatures import FunctionalTiedCenteredSAE as sig

    torch.manual_seed(16)
    d, n, B = 256, 512, 512
    models = [sig.init(d, n, l1, device=DEV) for l1 in (1e-4, 1e-3)]
    for p, _ in models:
        p["encoder_bias"].zero_()
        p["center"].normal_(0.0, 0.5)
    ref = FunctionalEnsemble([({k: v.clone() for k, v in p.items()}, b) for p, b in models], sig, adam,
                             {"lr": 1e-3}, device=DEV)
    fused = FusedSAEEnsemble(models, sig, lr=1e-3, batch_size=B, device=DEV)
    feats = torch.nn.functional.normalize(torch.randn(1024, d, device=DEV), dim=-1)
    x = ((torch.relu(torch.randn(B, 1024, device=DEV) - 1.0) * 2.0) @ feats + 0.3).to(torch.bfloat16)
    grads, _ = ref.compute_grads(x.float())
    ref.step_batch(x.float())
    out = fused.step_batch(x)
    torch.cuda.synchronize()
    assert float(out[:, 4].min()) > 0.3 * n, "codes must be dense for this test"
    # the gradient itself (from the PRE-update dictionary, as vmap(grad) in the reference)
    g_ref, g_fused = grads["center"].float(), fused.last_center_grad.float()
    for g in range(len(models)):
        rel = ((g_fused[g] - g_ref[g]).norm() / g_ref[g].norm()).item()
        assert rel < 5e-2, (g, rel)
    init = torch.stack([m[0]["center"] for m in models]).to(DEV)
    mf, mr = fused.params["center"] - init, ref.params["center"] - init
    big = mr.abs() > 0.5e-3  # Adam's first step: ~lr where the gradient is not tiny
    agree = (torch.sign(mf) == torch.sign(mr))[big].float().mean().item()
    assert agree > 0.9, agree


def test_synth_codes_kernel_statistics_and_reproducibility():
    """K17: Philox sparse codes -- per-feature firing rates match the probabilities, nonzero
    codes have mean E[U U] = 1/4, any row slice regenerates exactly, and the MFMA mixing GEMM
    matches fp32 matmul; the generator's hip backend produces data of the right shape/scale."""
    from sparse_coding__amd.data.synthetic import RandomDatasetGenerator
    from sparse_coding__amd.ops import synth

    n, B = 512, 65536
    probs = (0.999 ** torch.arange(n, device=DEV, dtype=torch.float32)) * (32.0 / n)
    c = synth.sparse_codes(probs, B, seed=1234)
    c2 = synth.sparse_codes(probs, B, seed=1234)
    assert torch.equal(c, c2)
    part = synth.sparse_codes(probs, 1000, seed=1234, row0=5000)
    assert torch.equal(part, c[5000:6000])
    assert not torch.equal(synth.sparse_codes(probs, 1000, seed=99), c[:1000])
    rate = (c != 0).float().mean(0)
    sd = (probs * (1 - probs) / B).sqrt()
    assert bool(((rate - probs).abs() <= 5 * sd + 1e-4).all())
    nz = c[c != 0].float()
    assert abs(nz.mean().item() - 0.25) < 0.01
    feats = torch.nn.functional.normalize(torch.randn(n, 256, device=DEV), dim=-1).to(torch.bfloat16)
    x = synth.mix(c[:4096], feats)
    ref = c[:4096].float() @ feats.float()
    torch.testing.assert_close(x.float(), ref, rtol=2e-2, atol=2e-2)
    gen = RandomDatasetGenerator(activation_dim=256, n_ground_truth_components=512, batch_size=2048,
                                 feature_num_nonzero=16, feature_prob_decay=0.99, correlated=False, device=DEV,
                                 seed=5, backend="hip")
    a, b = gen.send(None), gen.send(None)
    assert a.shape == (2048, 256) and not torch.equal(a, b) and torch.isfinite(a).all()
    genc = RandomDatasetGenerator(activation_dim=256, n_ground_truth_components=512, batch_size=2048,
                                  feature_num_nonzero=16, feature_prob_decay=0.99, correlated=True, device=DEV,
                                  seed=5, backend="hip")
    assert torch.isfinite(genc.send(None)).all()


@pytest.mark.parametrize("Gs,B,n,ks", [(2, 256, 1024, [3, 20]), (3, 2048, 6144, [8, 16, 24]), (1, 512, 256, [40])])
def test_topk_slot_lists_match_torch_sort(Gs, B, n, ks):
    """Device counting sort of the picks == a stable torch sort by (model, feature); the
    count buffer is left zeroed so the lists rebuild correctly on the next call."""
    from sparse_coding__amd.ops import topk as T

    torch.manual_seed(19)
    kmax = max(ks) + 4
    G = Gs + 1
    k = torch.tensor(ks + [kmax], dtype=torch.int32, device=DEV)
    lists = T.SlotLists(Gs, B, n, ks + [kmax], kmax, DEV)
    for rep in range(2):
        scores = torch.randn(G, B, n, device=DEV)
        scores[0, : B // 2, :5] = 9.0  # a few hot features: long lists
        idx, _ = T.topk_select(scores, k, kmax)
        T.slot_lists(idx, k, lists)
        torch.cuda.synchronize()
        assert int(lists.cnt.abs().sum()) == 0
        keys, slots = [], []
        for g in range(Gs):
            kg = ks[g]
            b = torch.arange(B, device=DEV).repeat_interleave(kg)
            s_ = torch.arange(kg, device=DEV).repeat(B)
            keys.append(g * n + idx[g, :, :kg].reshape(-1).long())
            slots.append((g * B + b) * kmax + s_)
        keys, slots = torch.cat(keys), torch.cat(slots)
        order = torch.sort(keys, stable=True).indices
        total = keys.numel()
        assert torch.equal(lists.perm[:total].long(), slots[order]), rep
        offs = torch.zeros(Gs * n + 1, dtype=torch.long, device=DEV)
        offs[1:] = torch.cumsum(torch.bincount(keys, minlength=Gs * n), 0)
        assert torch.equal(lists.offs.long(), offs), rep


@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
def test_topk_sparse_wgrad_matches_dense(out_dtype):
    """Slot-list weight gradient (small-k top-k models) == the dense GEMM over the scattered
    code / code-gradient buffers, on the same select + decode outputs."""
    from sparse_coding__amd.ops import gemm as GM
    from sparse_coding__amd.ops import topk as T

    torch.manual_seed(17)
    G, B, n, d = 3, 256, 1024, 256
    D = torch.nn.functional.normalize(torch.randn(G, n, d, device=DEV), dim=-1).to(torch.bfloat16)
    x = torch.randn(B, d, device=DEV).to(torch.bfloat16)
    ks = [3, 8, 20]
    k = torch.tensor(ks, dtype=torch.int32, device=DEV)
    scores = torch.empty(G, B, n, device=DEV)
    GM.matmul_nt(x, D, scores)
    idx, val = T.topk_select(scores, k, 20)
    r = torch.empty(G, B, d, device=DEV, dtype=torch.bfloat16)
    se = torch.empty(G, B, device=DEV)
    cb = torch.zeros(G, B, n, device=DEV, dtype=torch.bfloat16)
    db = torch.zeros(G, B, n, device=DEV, dtype=torch.bfloat16)
    dscv = torch.zeros(G, B, 20, device=DEV)
    T.decode_grad(idx, val, k, D, x, r, se, cb, db, dscv=dscv)
    dense = torch.empty(G, n, d, device=DEV)
    GM.weight_grads([[(cb, r), (db, x)]], [dense], 1e-2)
    lists = T.SlotLists(G, B, n, ks, 20, DEV)
    T.slot_lists(idx, k, lists)
    sparse = torch.empty(G, n, d, device=DEV, dtype=out_dtype)
    T.sparse_wgrad(lists, val, dscv, r, x, sparse, 1e-2)
    sparse2 = torch.empty(G, n, d, device=DEV, dtype=out_dtype)
    T.slot_lists(idx, k, lists)
    T.sparse_wgrad(lists, val, dscv, r, x, sparse2, 1e-2)
    # models below dense_from: the same dscv / residual, nothing scattered into the dense buffers
    cb2, db2, dscv2 = torch.zeros_like(cb), torch.zeros_like(db), torch.zeros_like(dscv)
    r2, se2 = torch.empty_like(r), torch.empty_like(se)
    T.decode_grad(idx, val, k, D, x, r2, se2, cb2, db2, dscv=dscv2, dense_from=2)
    torch.cuda.synchronize()
    assert torch.equal(dscv2, dscv) and torch.equal(r2, r) and torch.equal(se2, se)
    assert not cb2[:2].any() and not db2[:2].any()
    assert torch.equal(cb2[2:], cb[2:]) and torch.equal(db2[2:], db[2:])
    assert torch.equal(sparse, sparse2)  # deterministic
    for g in range(G):
        rel = ((sparse[g].float() - dense[g]).norm() / dense[g].norm()).item()
        assert rel < 1e-2, (g, rel)
    # rows nobody picked are exactly zero
    picked = torch.zeros(G, n, dtype=torch.bool, device=DEV)
    for g in range(G):
        picked[g, idx[g, :, : int(k[g])].reshape(-1).long()] = True
    assert float(sparse[~picked].float().abs().max()) == 0.0

