"""The row-block fused SAE forward (csrc/sae_rowblock.hip: encoder -> decoder -> code gradient in
one launch) against the three separate GEMM kernels and a plain PyTorch fp32 reference."""

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from sparse_coding__amd.ops import _lib as L

    L.lib()  # must load: no silent fallback on a GPU box
    yield


def _rel(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _run_rowblock(x, we, wd, bias, l1, count=True):
    from sparse_coding__amd.ops import gemm

    G, n, d = we.shape
    B = x.shape[-2]
    bf = torch.bfloat16
    out = dict(c=torch.empty(G, B, n, device=DEV, dtype=bf), r=torch.empty(G, B, d, device=DEV, dtype=bf),
               dpre=torch.empty(G, B, n, device=DEV, dtype=bf),
               mask=torch.zeros(gemm.code_mask_shape(G, B, n), device=DEV, dtype=torch.int64),
               enc=torch.full((G, B // 64, 2), float("nan"), device=DEV),
               dec=torch.full((G, B // 64), float("nan"), device=DEV),
               col=torch.full((G, B // 32, n), float("nan"), device=DEV),
               cnt=torch.full((G, B // 32, n), float("nan"), device=DEV) if count else None)
    gemm.sae_forward_rowblock(x, we, wd, bias, l1, out["c"], out["r"], out["dpre"], out["mask"], out["enc"],
                              out["dec"], out["col"], out["cnt"])
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("G,B,n,shared_x", [(3, 256, 256, True), (2, 128, 1024, False), (8, 2048, 2048, True),
                                            (1, 64, 512, True)])
def test_rowblock_matches_separate_kernels_and_fp32(G, B, n, shared_x):
    from sparse_coding__amd.ops import gemm

    torch.manual_seed(7)
    d = 512
    x = (torch.randn(B, d, device=DEV) if shared_x else torch.randn(G, B, d, device=DEV)).to(torch.bfloat16)
    we = (torch.randn(G, n, d, device=DEV) * 0.05).to(torch.bfloat16)
    wd = torch.nn.functional.normalize(torch.randn(G, n, d, device=DEV), dim=-1).to(torch.bfloat16)
    bias = torch.randn(G, n, device=DEV) * 0.1 - 0.05
    l1 = torch.logspace(-4, -2, G, device=DEV)
    o = _run_rowblock(x, we, wd, bias, l1)

    # the three separate kernels on the same inputs
    c = torch.empty_like(o["c"])
    part = torch.zeros(G, (B // 128 or 1) * (n // 128), 2, device=DEV)
    cmask = torch.zeros_like(o["mask"])
    if B % 128 == 0:
        cnt = torch.zeros(G, B // 128, n, device=DEV)
        gemm.encode_relu(x, we, bias, c, part, cnt, None, mask_out=cmask)
        r = torch.empty_like(o["r"])
        dpart = torch.zeros(G, (B // 128) * (d // 128), device=DEV)
        gemm.decode_residual(c, wd, x, r, dpart)
        dpre = torch.empty_like(o["dpre"])
        colpart = torch.zeros(G, B // 128, n, device=DEV)
        gemm.code_grad(r, wd, c, l1, dpre, colpart, mask=cmask)
        torch.cuda.synchronize()
        # same operands, same K order, same rounding points: the codes and mask are identical
        assert torch.equal(o["c"], c)
        assert torch.equal(o["mask"], cmask)
        assert _rel(o["r"], r) < 2e-3
        assert _rel(o["dpre"], dpre) < 5e-3
        torch.testing.assert_close(o["col"].sum(1), colpart.sum(1), rtol=1e-3, atol=1e-2)
        torch.testing.assert_close(o["cnt"].sum(1), cnt.sum(1), rtol=0, atol=0)
        torch.testing.assert_close(o["enc"].sum(1), part.sum(1), rtol=1e-4, atol=1e-2)
        torch.testing.assert_close(o["dec"].sum(1), dpart.sum(1), rtol=1e-3, atol=1e-2)

    # fp32 reference (from the kernel's own bf16 codes / residual, the rounding points of the step)
    xs = x.float() if x.dim() == 3 else x.float().expand(G, B, d)
    pre = xs @ we.float().transpose(1, 2) + bias[:, None, :]
    cref = torch.relu(pre)
    assert _rel(o["c"], cref) < 1e-2
    cf = o["c"].float()
    rref = cf @ wd.float() - xs
    assert _rel(o["r"], rref) < 1e-2
    dref = (o["r"].float() @ wd.float().transpose(1, 2) + (l1 * d / 2)[:, None, None]) * (cf > 0)
    assert _rel(o["dpre"], dref) < 1e-2
    torch.testing.assert_close(o["enc"][..., 0].sum(1), cf.sum((1, 2)), rtol=1e-2, atol=1e-1)
    torch.testing.assert_close(o["enc"][..., 1].sum(1), (cf > 0).float().sum((1, 2)), rtol=0, atol=0)
    torch.testing.assert_close(o["dec"].sum(1), (rref ** 2).sum((1, 2)), rtol=2e-2, atol=1e-1)
    torch.testing.assert_close(o["col"].sum(1), dref.sum(1), rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(o["cnt"].sum(1), (cf > 0).float().sum(1), rtol=0, atol=0)


@pytest.mark.parametrize("kind", ["untied", "tied"])
def test_fused_engine_rowblock_matches_separate_kernels(kind):
    """Five Adam steps of the engine with the row-block forward and with the three GEMMs."""
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.models.signatures import FunctionalSAE, FunctionalTiedSAE

    torch.manual_seed(11)
    sig = FunctionalSAE if kind == "untied" else FunctionalTiedSAE
    d, n, B = 512, 1024, 512
    models = [sig.init(d, n, l1, device=DEV) for l1 in (1e-4, 1e-3, 1e-2)]
    a = FusedSAEEnsemble(models, sig, lr=1e-3, batch_size=B, device=DEV, rowblock=True, count_every=2)
    b = FusedSAEEnsemble(models, sig, lr=1e-3, batch_size=B, device=DEV, rowblock=False, count_every=2)
    assert a.rowblock and not b.rowblock
    feats = torch.nn.functional.normalize(torch.randn(2048, d, device=DEV), dim=-1)
    for _ in range(5):
        x = (torch.relu(torch.randn(B, 2048, device=DEV) - 2.0) @ feats).to(torch.bfloat16)
        oa = a.step_batch(x).clone()
        ob = b.step_batch(x).clone()
        torch.cuda.synchronize()
        torch.testing.assert_close(oa, ob, rtol=2e-3, atol=1e-5)
    for k in a.params:
        assert _rel(a.params[k] - torch.stack([m[0][k] for m in models]),
                    b.params[k] - torch.stack([m[0][k] for m in models])) < 2e-2, k
    torch.testing.assert_close(a.feature_counts, b.feature_counts, rtol=0, atol=0)


def test_rowblock_graph_replay_matches_eager():
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.models.signatures import FunctionalSAE

    torch.manual_seed(4)
    d, n, B = 512, 2048, 2048
    models = [FunctionalSAE.init(d, n, l1, device=DEV) for l1 in (1e-4, 1e-3, 3e-3, 1e-2)]
    eager = FusedSAEEnsemble(models, FunctionalSAE, batch_size=B, device=DEV, rowblock=True)
    graph = FusedSAEEnsemble(models, FunctionalSAE, batch_size=B, device=DEV, rowblock=True).enable_graph()
    assert eager.rowblock and graph.rowblock
    for _ in range(3):
        x = torch.randn(B, d, device=DEV).to(torch.bfloat16)
        eager.step_batch(x)
        graph.step_batch(x)
    torch.cuda.synchronize()
    for k in eager.params:
        torch.testing.assert_close(graph.params[k], eager.params[k], rtol=0, atol=0)
    torch.testing.assert_close(graph.out, eager.out, rtol=0, atol=0)


def test_in_graph_ring_source_matches_host_sampling():
    """Batch fetch inside the step's HIP graph (DeviceRing.graph_source, indexed by the device
    step counter) == host-driven sampling + graph replay, across permutation (epoch) rollovers."""
    from sparse_coding__amd.data.ring import DeviceRing
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.models.signatures import FunctionalSAE

    torch.manual_seed(9)
    d, n, B = 512, 1024, 256
    rows = (torch.randn(B * 7 // 2, d, device=DEV) * 2).to(torch.bfloat16)  # 3.5 batches: 3-step epochs
    rings = []
    for _ in range(2):
        r = DeviceRing(rows.shape[0], d, device=DEV, seed=5)
        r.push(rows)
        rings.append(r)
    models = [FunctionalSAE.init(d, n, l1, device=DEV) for l1 in (1e-4, 1e-3)]
    a = FusedSAEEnsemble(models, FunctionalSAE, batch_size=B, device=DEV).enable_graph()
    a.attach_source(rings[0].graph_source(B))
    b = FusedSAEEnsemble(models, FunctionalSAE, batch_size=B, device=DEV).enable_graph()
    for _ in range(8):
        a.step_source()
        rings[1].sample_shard(B, 0, 1, out=b.x_static)
        b.step_static()
    torch.cuda.synchronize()
    assert rings[0].epoch == rings[1].epoch >= 3
    torch.testing.assert_close(a.x_static, b.x_static, rtol=0, atol=0)
    for k in a.params:
        torch.testing.assert_close(a.params[k], b.params[k], rtol=0, atol=0)


@pytest.mark.parametrize("group", [8, 3])
def test_multi_step_graph_replay_matches_single_steps(group):
    """``step_source(k)``: k optimizer steps (batch gathers included) in ONE graph replay equal k
    single-step replays on host-sampled batches: parameters, losses, feature counts."""
    from sparse_coding__amd.data.ring import DeviceRing
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.models.signatures import FunctionalSAE

    torch.manual_seed(10)
    d, n, B, steps = 512, 1024, 256, 16
    rows = (torch.randn(B * 40, d, device=DEV) * 2).to(torch.bfloat16)
    rings = []
    for _ in range(2):
        r = DeviceRing(rows.shape[0], d, device=DEV, seed=3)
        r.push(rows)
        rings.append(r)
    models = [FunctionalSAE.init(d, n, l1, device=DEV) for l1 in (1e-4, 1e-3, 1e-2)]
    a = FusedSAEEnsemble(models, FunctionalSAE, batch_size=B, device=DEV).enable_graph()
    a.attach_source(rings[0].graph_source(B))
    b = FusedSAEEnsemble(models, FunctionalSAE, batch_size=B, device=DEV).enable_graph()
    done = 0
    while done < steps:
        k = min(group, steps - done)
        a.step_source(k)
        done += k
    for _ in range(steps):
        rings[1].sample_shard(B, 0, 1, out=b.x_static)
        b.step_static()
    torch.cuda.synchronize()
    assert a.step_count == b.step_count == steps and int(a.step_dev.item()) == steps
    for k in a.params:
        torch.testing.assert_close(a.params[k], b.params[k], rtol=0, atol=0)
    torch.testing.assert_close(a.out, b.out, rtol=0, atol=0)
    torch.testing.assert_close(a.feature_counts, b.feature_counts, rtol=0, atol=0)
    assert a.rows_seen == b.rows_seen


def test_prime_source_captures_without_running():
    """``prime_source`` captures the group / single-step graphs at the current step without
    executing any step (parameters and counters unchanged); later replays reuse them."""
    from sparse_coding__amd.data.ring import DeviceRing
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.models.signatures import FunctionalSAE

    torch.manual_seed(12)
    d, n, B = 512, 512, 256
    ring = DeviceRing(B * 20, d, device=DEV, seed=1)
    ring.push((torch.randn(B * 20, d, device=DEV)).to(torch.bfloat16))
    models = [FunctionalSAE.init(d, n, 1e-3, device=DEV)]
    e = FusedSAEEnsemble(models, FunctionalSAE, batch_size=B, device=DEV).enable_graph()
    e.attach_source(ring.graph_source(B))
    e.step_source(1)
    e.step_source(1)
    torch.cuda.synchronize()
    before = {k: v.clone() for k, v in e.params.items()}
    e.prime_source(8)
    torch.cuda.synchronize()
    n_graphs = len(e._graph)
    assert e.step_count == 2 and int(e.step_dev.item()) == 2
    for k in before:
        assert torch.equal(before[k], e.params[k])
    e.step_source(8)
    e.step_source(1)
    torch.cuda.synchronize()
    assert len(e._graph) == n_graphs and e.step_count == 11 and int(e.step_dev.item()) == 11
