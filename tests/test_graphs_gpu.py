"""HIP graph replays of the fused step: the in-graph ring batch fetch, multi-step graphs (k optimizer
steps per replay) and priming (capture + upload without running), against host-driven steps."""

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from sparse_coding__amd.ops import _lib as L

    L.lib()  # must load: no silent fallback on a GPU box
    yield


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


@pytest.mark.parametrize("kind,G,B", [("untied", 3, 256), ("tied", 3, 256), ("untied", 1, 4096)])
def test_fused_step_tail_matches_separate_kernels(kind, G, B, monkeypatch):
    """The fused step tail (row Adam + loss terms + bias Adam + step counter in one launch, |b| from
    parity-double-buffered b^2 partials) against the separate adam_rows / loss_reduce / bias_adam
    kernels: parameters, moments, losses, feature counts and the device step counter, over eager steps
    (counting and non-counting) with a non-zero bias decay, and after an out-of-band bias edit."""
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.models.signatures import FunctionalSAE, FunctionalTiedSAE

    torch.manual_seed(21)
    sig = FunctionalSAE if kind == "untied" else FunctionalTiedSAE
    d, n = 512, 1024
    hp = ((1e-3, 1e-3), (1e-4, 0.0), (1e-2, 3e-2))[:G]
    models = [sig.init(d, n, l1, bias_decay=bd, device=DEV) for l1, bd in hp]
    for p, _ in models:
        p["encoder_bias"].normal_(0.0, 0.1)
    a = FusedSAEEnsemble(models, sig, lr=1e-3, batch_size=B, device=DEV, count_every=2)
    monkeypatch.setenv("SC_FUSED_TAIL", "0")
    b = FusedSAEEnsemble(models, sig, lr=1e-3, batch_size=B, device=DEV, count_every=2)
    assert a._tail_ok and not b._tail_ok
    assert (a.wsplit > 1) == (G == 1)  # one model on a large batch: split-K gradient slabs into the tail
    feats = torch.nn.functional.normalize(torch.randn(2048, d, device=DEV), dim=-1)
    for i in range(6):
        if i == 3:  # an out-of-band edit of the bias (refresh_shadows marks the b^2 partials stale)
            for e in (a, b):
                e.params["encoder_bias"].mul_(0.5)
                e.refresh_shadows()
        x = (torch.relu(torch.randn(B, 2048, device=DEV) - 2.0) @ feats).to(torch.bfloat16)
        oa = a.step_batch(x).clone()
        ob = b.step_batch(x).clone()
        torch.cuda.synchronize()
        torch.testing.assert_close(oa, ob, rtol=1e-5, atol=1e-6)
    assert int(a.step_dev.item()) == int(b.step_dev.item()) == 6 and int(a._ticket.abs().sum().item()) == 0
    # (|b| is summed in another order -- per-32-column partials -- so the bias-decay gradient, and
    # through the codes everything downstream, may differ in the last bits)
    for k in a.params:
        torch.testing.assert_close(a.params[k], b.params[k], rtol=1e-4, atol=2e-6)
        torch.testing.assert_close(a.m[k], b.m[k], rtol=1e-3, atol=1e-8)
        torch.testing.assert_close(a.v[k], b.v[k], rtol=1e-3, atol=1e-11)
    torch.testing.assert_close(a.feature_counts, b.feature_counts, rtol=0, atol=0)


@pytest.mark.parametrize("mode,chunks", [("dp", 1), ("dp", 2), ("zero1", 2)])
def test_graphed_data_parallel_one_rank_matches_single_engine(mode, chunks):
    """Data parallel with the collectives captured in multi-step graphs (native RCCL communicator on
    its own stream, one rank) == the single-engine multi-step graph on the same ring batches:
    parameters, losses and feature counts (model chunks, cross-step update order, ZeRO-1 shards)."""
    from sparse_coding__amd.data.ring import DeviceRing
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.engine.graph_plan import count_pattern
    from sparse_coding__amd.models.signatures import FunctionalSAE
    from sparse_coding__amd.parallel.data_parallel import split_models
    from sparse_coding__amd.parallel.dist import DistInfo
    from sparse_coding__amd.parallel.graphed import GraphedDataParallel
    from sparse_coding__amd.parallel.rccl import RcclComm

    torch.manual_seed(17)
    d, n, B = 512, 1024, 256
    rows = (torch.randn(B * 40, d, device=DEV) * 2).to(torch.bfloat16)
    rings = []
    for _ in range(2):
        r = DeviceRing(rows.shape[0], d, device=DEV, seed=6)
        r.push(rows)
        rings.append(r)
    models = [FunctionalSAE.init(d, n, l1, device=DEV) for l1 in (1e-4, 1e-3, 3e-3, 1e-2)]
    info = DistInfo(device=torch.device(DEV))
    comm = RcclComm(info)
    engines = [FusedSAEEnsemble(m, FunctionalSAE, lr=1e-3, batch_size=B, device=DEV) for m in split_models(models, chunks)]
    gdp = GraphedDataParallel(engines, info, comm, rings[0].graph_source(B), mode=mode)
    single = FusedSAEEnsemble(models, FunctionalSAE, lr=1e-3, batch_size=B, device=DEV).enable_graph()
    single.attach_source(rings[1].graph_source(B))
    for s in (3, 5, 3):
        gdp.run(s, count_pattern(s))
        single.step_source(s, count_pattern(s))
    torch.cuda.synchronize()
    comm.close()
    # (the two paths sum the gradients in different orders -- one- vs two-problem weight-gradient
    # launches, bias sums in torch vs in the fused tail -- and Adam amplifies last-bit differences of
    # near-zero gradients, so compare the parameter CHANGES in norm)
    for k in single.params:
        got = torch.cat([e.params[k] for e in engines])
        p0 = torch.stack([m[0][k] for m in models])
        rel = float((got - single.params[k]).norm() / (single.params[k] - p0).norm())
        assert rel < 1e-2, (k, rel)
    # feature on-counts: every counting step's rows (a handful of codes near zero may flip with the
    # last-bit parameter differences)
    dc = (torch.cat([e.feature_counts for e in engines]) - single.feature_counts).abs()
    assert float(dc.max()) <= 2 and float((dc > 0).float().mean()) < 0.01, (float(dc.max()), float((dc > 0).float().mean()))
    assert float(single.feature_counts.sum()) > 0
    torch.testing.assert_close(torch.cat([e.out for e in engines])[:, :3], single.out[:, :3], rtol=1e-3, atol=1e-6)
    assert all(int(e.step_dev.item()) == 11 for e in engines)


def test_graphed_ensemble_sharded_one_rank_matches_single_engine():
    """Ensemble sharding with the batch fetch and the in-place all-gathers captured in the group graph
    (native RCCL communicator, one rank) == the single-engine multi-step graph on the same ring
    batches: the same kernels on the same rows, so parameters and losses agree exactly."""
    from sparse_coding__amd.data.ring import DeviceRing
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.engine.graph_plan import count_pattern
    from sparse_coding__amd.models.signatures import FunctionalSAE
    from sparse_coding__amd.parallel.dist import DistInfo
    from sparse_coding__amd.parallel.ensemble_shard import EnsembleSharded
    from sparse_coding__amd.parallel.graphed import GraphedEnsembleSharded
    from sparse_coding__amd.parallel.rccl import RcclComm

    torch.manual_seed(23)
    d, n, B = 512, 1024, 256
    rows = (torch.randn(B * 40, d, device=DEV) * 2).to(torch.bfloat16)
    rings = []
    for _ in range(2):
        r = DeviceRing(rows.shape[0], d, device=DEV, seed=8)
        r.push(rows)
        rings.append(r)
    models = [FunctionalSAE.init(d, n, l1, device=DEV) for l1 in (1e-4, 1e-3, 3e-3, 1e-2)]
    info = DistInfo(device=torch.device(DEV))
    comm = RcclComm(info)
    es = EnsembleSharded(models, lambda m, bs: FusedSAEEnsemble(m, FunctionalSAE, lr=1e-3, batch_size=bs, device=DEV),
                         info, batch_per_rank=B, d=d)
    ges = GraphedEnsembleSharded(es, comm, rings[0].graph_source(B, 0, 1))
    ges.prime([count_pattern(s) for s in (3, 5)])
    single = FusedSAEEnsemble(models, FunctionalSAE, lr=1e-3, batch_size=B, device=DEV).enable_graph()
    single.attach_source(rings[1].graph_source(B))
    for s in (3, 5, 3, 5):
        ges.run(s, count_pattern(s))
        single.step_source(s, count_pattern(s))
    torch.cuda.synchronize()
    comm.close()
    for k in single.params:
        torch.testing.assert_close(es.engine.params[k], single.params[k], rtol=0, atol=0)
    torch.testing.assert_close(es.engine.out, single.out, rtol=0, atol=0)
    torch.testing.assert_close(es.engine.feature_counts, single.feature_counts, rtol=0, atol=0)
    assert int(es.engine.step_dev.item()) == 16


@pytest.mark.parametrize("mode", ["dp", "zero1"])
def test_trainer_graphed_data_parallel_one_rank(mode):
    """EnsembleTrainer(parallel='dp' / 'zero1') on a GPU: the fused engine with in-graph RCCL
    collectives (one rank, caller-provided batches) trains like the plain fused trainer."""
    from sparse_coding__amd.engine.trainer import EnsembleTrainer
    from sparse_coding__amd.models.signatures import FunctionalSAE
    from sparse_coding__amd.parallel.dist import DistInfo

    torch.manual_seed(19)
    d, n, B = 512, 1024, 256
    models = [FunctionalSAE.init(d, n, l1, device=DEV) for l1 in (1e-4, 1e-3, 1e-2)]
    tr = EnsembleTrainer(models, FunctionalSAE, lr=1e-3, batch_size=B, device=DEV, parallel=mode,
                         dist=DistInfo(device=torch.device(DEV)), args={"dict_size": n})
    ref = EnsembleTrainer(models, FunctionalSAE, lr=1e-3, batch_size=B, device=DEV, args={"dict_size": n})
    assert tr.kind == f"{mode}-graphed" and ref.kind == "fused-sae"
    feats = torch.nn.functional.normalize(torch.randn(2048, d, device=DEV), dim=-1)
    for _ in range(6):
        x = (torch.relu(torch.randn(B, 2048, device=DEV) - 2.0) @ feats).to(torch.bfloat16)
        a = tr.step(x).clone()
        b = ref.step(x).clone()
    torch.cuda.synchronize()
    torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-6)
    for k in ref.impl.params:
        p0 = torch.stack([m[0][k] for m in models])
        rel = float((tr.impl.params[k] - ref.impl.params[k]).norm() / (ref.impl.params[k] - p0).norm())
        assert rel < 1e-2, (k, rel)
    lds = tr.to_learned_dicts(["dict_size"], ["l1_alpha"])
    assert len(lds) == 3 and lds[2][1]["dict_size"] == n
    st = tr.state_dict()
    assert st["kind"] == f"{mode}-graphed" and st["impl"]["step"] == 6


@pytest.mark.parametrize("sig_name,mode", [("FunctionalMaskedTiedSAE", "dp"), ("FunctionalMaskedSAE", "dp"),
                                           ("FunctionalMaskedSAE", "zero1")])
def test_trainer_graphed_data_parallel_masked_one_rank(sig_name, mode):
    """Masked ensembles (models of different live sizes stacked to one width, the reference's
    dict_ratio experiment, big_sweep_experiments.py:546-580) train data-parallel on the graphed path:
    EnsembleTrainer(parallel='dp' / 'zero1') at one RCCL rank == the plain fused masked trainer, and
    the dead rows / columns stay exactly as initialised."""
    from sparse_coding__amd.engine.trainer import EnsembleTrainer
    from sparse_coding__amd.models import signatures as S
    from sparse_coding__amd.parallel.dist import DistInfo

    sig = getattr(S, sig_name)
    torch.manual_seed(43)
    d, n, B = 512, 1024, 256
    sizes = (256, 512, 768, 1024)
    models = [sig.init(d, sz, n, l1, device=DEV) for sz, l1 in zip(sizes, (1e-4, 1e-3, 3e-3, 1e-2))]
    tr = EnsembleTrainer(models, sig, lr=1e-3, batch_size=B, device=DEV, parallel=mode,
                         dist=DistInfo(device=torch.device(DEV)), args={"dict_size": n})
    ref = EnsembleTrainer(models, sig, lr=1e-3, batch_size=B, device=DEV, args={"dict_size": n})
    assert tr.kind == f"{mode}-graphed" and ref.kind == "fused-sae" and tr.impl.nactive is not None
    feats = torch.nn.functional.normalize(torch.randn(2048, d, device=DEV), dim=-1)
    for _ in range(6):
        x = (torch.relu(torch.randn(B, 2048, device=DEV) - 2.0) @ feats).to(torch.bfloat16)
        a = tr.step(x).clone()
        b = ref.step(x).clone()
    torch.cuda.synchronize()
    tr.close()
    torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-6)
    for k in ref.impl.params:
        p0 = torch.stack([m[0][k] for m in models])
        rel = float((tr.impl.params[k] - ref.impl.params[k]).norm() / (ref.impl.params[k] - p0).norm())
        assert rel < 1e-2, (k, rel)
        for g, sz in enumerate(sizes):  # dead rows never move
            assert torch.equal(tr.impl.params[k][g, sz:], p0[g, sz:]), (k, g)
    lds = tr.to_learned_dicts(["dict_size"], ["l1_alpha"])
    assert [ld.n_feats for ld, _ in lds] == list(sizes)


def test_ring_gather_into_global_matches_indexing():
    """One launch fills rank r's slots of s consecutive global batches from the ring permutation
    (the in-place all-gather layout of graphed ensemble sharding); other ranks' slots untouched."""
    from sparse_coding__amd.data.ring import DeviceRing

    torch.manual_seed(29)
    d, B, N, r, s = 256, 64, 3, 1, 4
    rows = (torch.randn(B * N * 12, d, device=DEV)).to(torch.bfloat16)
    ring = DeviceRing(rows.shape[0], d, device=DEV, seed=3)
    ring.push(rows)
    src = ring.graph_source(B, r, N)
    src.prepare(2, s)
    step = torch.tensor([4], device=DEV, dtype=torch.int32)
    glob = torch.zeros(s, N * B, d, device=DEV, dtype=torch.bfloat16)
    src.gather_into_global(glob, step)
    t0 = (4 - int(src.ep0.item())) * N * B
    for k in range(s):
        idx = src.perm[t0 + k * N * B + r * B: t0 + k * N * B + (r + 1) * B]
        assert torch.equal(glob[k, r * B:(r + 1) * B], ring.buf[idx])
        assert not glob[k, :r * B].any() and not glob[k, (r + 1) * B:].any()


def test_topk_multistep_source_graph_matches_eager_steps():
    """Top-k engine: odd / even multi-step graphs with the batch gather inside (run_source) are
    bit-identical to eager steps on the same permutation's batches."""
    from sparse_coding__amd.data.ring import DeviceRing
    from sparse_coding__amd.engine.topk import FusedTopKEnsemble
    from sparse_coding__amd.models.topk import TopKEncoder

    torch.manual_seed(31)
    d, n, B, ks = 256, 1024, 256, [4, 8, 32]
    models = [TopKEncoder.init(d, n, k, device=DEV) for k in ks]
    a = FusedTopKEnsemble(models, lr=1e-3, batch_size=B, device=DEV)
    b = FusedTopKEnsemble(models, lr=1e-3, batch_size=B, device=DEV)
    rows = torch.randn(B * 16, d, device=DEV).to(torch.bfloat16)
    ring = DeviceRing(rows.shape[0], d, device=DEV, seed=5)
    ring.push(rows)
    src = ring.graph_source(B)
    losses_a = []
    for s in (3, 2, 3):
        a.run_source(src, s)
        losses_a.append(a.mse.clone())
    assert a.step_count == 8 and int(src.ep0.item()) == 0
    losses_b = []
    for t in range(8):
        b.step_batch(ring.buf[src.perm[t * B:(t + 1) * B]])
        if t in (2, 4, 7):
            losses_b.append(b.mse.clone())
    torch.cuda.synchronize()
    for la, lb in zip(losses_a, losses_b):
        assert torch.equal(la, lb)
    assert torch.equal(a.params["dict"], b.params["dict"])
    assert torch.equal(a.idx, b.idx)

