"""Stream ordering of the in-graph multi-GPU steps on ONE GPU (``parallel/sim_comm.DelayedSimComm``).

At one RCCL rank every collective lands almost at once, and the gloo rehearsal communicator is
synchronous, so neither can show a consumer that forgot to wait for a collective's event.  Here the
graphed data-parallel and ensemble-sharded steps are CAPTURED on a communicator whose collectives run
on their own stream behind a 50 us spin kernel and simulate 2 identical replicas (all-reduce x2,
all-gather copies this rank's block everywhere), and compared bitwise against the same sequence run
eagerly with every collective on the current stream (fully ordered).

Mutation check (run in-test, every time): the same capture with the joins removed -- the data-parallel
``GraphedDataParallel._wait`` replaced by a no-op (the update then reads the gradient before its
all-reduce lands), the ensemble-sharded gathers returning no event (step k then copies its global
batch before the gather filled it) -- must NOT match.  Deleting the ``_wait(c.red_ev)`` in
``GraphedDataParallel._update`` or either ``cur.wait_event`` of ``GraphedEnsembleSharded._steps``
(parallel/graphed.py) is therefore caught.  ZeRO-1's shard gathers are not simulated faithfully
(other ranks own other rows) and stay with the multi-rank gloo tests.

These tests found a HIP graph-capture bug: with one comm-stream fork per collective, the first
capturing-stream node after five or more consecutive forks lost its dependency and ran unordered across
replays; the graphed classes now fork once per batch of collectives (profiles/r6/graph_capture/).
"""

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from sparse_coding__amd.ops import _lib as L

    L.lib()  # must load: no silent fallback on a GPU box
    yield


def _rings(d, B, seed, copies=3):
    from sparse_coding__amd.data.ring import DeviceRing

    torch.manual_seed(seed)
    rows = (torch.randn(B * 48, d, device=DEV) * 2).to(torch.bfloat16)
    out = []
    for _ in range(copies):
        r = DeviceRing(rows.shape[0], d, device=DEV, seed=seed)
        r.push(rows)
        out.append(r)
    return out


def _dp(models, chunks, comm, ring, B, capture, world=2):
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.models.signatures import FunctionalSAE
    from sparse_coding__amd.parallel.data_parallel import split_models
    from sparse_coding__amd.parallel.dist import DistInfo
    from sparse_coding__amd.parallel.graphed import GraphedDataParallel

    info = DistInfo(rank=0, world_size=world, device=torch.device(DEV))
    engines = [FusedSAEEnsemble(m, FunctionalSAE, lr=1e-3, batch_size=B, device=DEV) for m in split_models(models, chunks)]
    gdp = GraphedDataParallel(engines, info, comm, ring.graph_source(B, 0, world), mode="dp", capture=capture)
    return gdp, engines


def _run_dp(gdp, groups=(3, 5, 3)):
    from sparse_coding__amd.engine.graph_plan import count_pattern

    gdp.prime([count_pattern(s) for s in sorted(set(groups))])
    for s in groups:
        gdp.run(s, count_pattern(s))
    torch.cuda.synchronize()


def _same(a_engines, b_engines):
    return all(torch.equal(a.params[k], b.params[k]) and torch.equal(a.m[k], b.m[k])
               for a, b in zip(a_engines, b_engines) for k in a.params) and all(
        torch.equal(a.out, b.out) for a, b in zip(a_engines, b_engines))


@pytest.mark.parametrize("chunks", [1, 2])
def test_graphed_dp_on_delayed_comm_matches_ordered_run(chunks, monkeypatch):
    """Data parallel (2 simulated replicas, ``chunks`` model chunks, the last chunk's update crossing
    into the next step) captured on the delayed communicator == the fully ordered eager run, bitwise;
    without the joins it differs."""
    from sparse_coding__amd.models.signatures import FunctionalSAE
    from sparse_coding__amd.parallel.graphed import GraphedDataParallel
    from sparse_coding__amd.parallel.sim_comm import DelayedSimComm

    d, n, B = 512, 1024, 256
    rings = _rings(d, B, 31)
    models = [FunctionalSAE.init(d, n, l1, device=DEV) for l1 in (1e-4, 1e-3, 3e-3, 1e-2)]
    ref, ref_e = _dp(models, chunks, DelayedSimComm(DEV, world=2, delay_us=0, sync=True), rings[0], B, capture=False)
    _run_dp(ref)
    comm = DelayedSimComm(DEV, world=2, delay_us=50)
    got, got_e = _dp(models, chunks, comm, rings[1], B, capture=True)
    _run_dp(got)
    assert comm.calls.get("all_reduce", 0) >= chunks  # the collectives were captured on the delayed stream
    assert _same(got_e, ref_e)
    assert all(int(e.step_dev.item()) == 11 for e in got_e)
    # the sensitivity of this comparison: the same capture without the joins does not match
    monkeypatch.setattr(GraphedDataParallel, "_wait", lambda self, evs: None)
    bad, bad_e = _dp(models, chunks, DelayedSimComm(DEV, world=2, delay_us=50), rings[2], B, capture=True)
    _run_dp(bad)
    assert not _same(bad_e, ref_e), "a missing wait on the all-reduce event went unnoticed"


def test_graphed_dp_on_simulated_replicas_is_one_rank_training():
    """The simulation's semantics: 2 identical replicas all-reduce to 2x the gradient and the engines
    scale it by 1/2, so the data-parallel update equals one engine trained on rank 0's rows."""
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.engine.graph_plan import count_pattern
    from sparse_coding__amd.models.signatures import FunctionalSAE
    from sparse_coding__amd.parallel.sim_comm import DelayedSimComm

    d, n, B = 512, 1024, 256
    rings = _rings(d, B, 37, copies=2)
    models = [FunctionalSAE.init(d, n, l1, device=DEV) for l1 in (1e-4, 1e-2)]
    gdp, engines = _dp(models, 1, DelayedSimComm(DEV, world=2, delay_us=20), rings[0], B, capture=True)
    _run_dp(gdp, (3, 5))
    single = FusedSAEEnsemble(models, FunctionalSAE, lr=1e-3, batch_size=B, device=DEV).enable_graph()
    single.attach_source(rings[1].graph_source(B, 0, 2))  # rank 0's shard of the same permutation
    for s in (3, 5):
        single.step_source(s, count_pattern(s))
    torch.cuda.synchronize()
    for k in single.params:
        p0 = torch.stack([m[0][k] for m in models])
        rel = float((engines[0].params[k] - single.params[k]).norm() / (single.params[k] - p0).norm())
        assert rel < 1e-2, (k, rel)


class _NoEventGather:
    """Wraps a comm so its all-gathers return no event: the consumer has nothing to wait on."""

    def __init__(self, comm):
        self._c = comm

    def __getattr__(self, k):
        return getattr(self._c, k)

    def all_gather(self, out, inp, overlap=False, fork=True):
        self._c.all_gather(out, inp, overlap=overlap, fork=fork)
        return None


def _es(models, comm, ring, B, d, capture, world=2):
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.models.signatures import FunctionalSAE
    from sparse_coding__amd.parallel.dist import DistInfo
    from sparse_coding__amd.parallel.ensemble_shard import EnsembleSharded
    from sparse_coding__amd.parallel.graphed import GraphedEnsembleSharded

    info = DistInfo(rank=0, world_size=world, device=torch.device(DEV))
    es = EnsembleSharded(models, lambda m, bs: FusedSAEEnsemble(m, FunctionalSAE, lr=1e-3, batch_size=bs, device=DEV),
                         info, batch_per_rank=B, d=d)
    return GraphedEnsembleSharded(es, comm, ring.graph_source(B, 0, world), capture=capture), es


def _run_es(ges, groups=(3, 10, 5)):  # (10: the bench's group size -- 10 collectives per group graph)
    from sparse_coding__amd.engine.graph_plan import count_pattern

    ges.prime([count_pattern(s) for s in sorted(set(groups))])
    for s in groups:
        ges.run(s, count_pattern(s))
    torch.cuda.synchronize()


def test_graphed_es_on_delayed_comm_matches_ordered_run():
    """Ensemble sharding (2 simulated replicas: rank 0 trains half the models on a 2B-row global batch)
    captured on the delayed communicator == the fully ordered eager run, bitwise; with the gathers'
    events dropped it differs."""
    from sparse_coding__amd.models.signatures import FunctionalSAE
    from sparse_coding__amd.parallel.sim_comm import DelayedSimComm

    d, n, B = 512, 1024, 256
    rings = _rings(d, B, 41)
    models = [FunctionalSAE.init(d, n, l1, device=DEV) for l1 in (1e-4, 1e-3, 3e-3, 1e-2)]
    ref, ref_es = _es(models, DelayedSimComm(DEV, world=2, delay_us=0, sync=True), rings[0], B, d, capture=False)
    _run_es(ref)
    comm = DelayedSimComm(DEV, world=2, delay_us=50)
    got, got_es = _es(models, comm, rings[1], B, d, capture=True)
    _run_es(got)
    assert comm.calls.get("all_gather", 0) >= 10
    assert got_es.engine.n_models == 2
    assert _same([got_es.engine], [ref_es.engine])
    torch.testing.assert_close(got._glob, ref._glob, rtol=0, atol=0)
    bad, bad_es = _es(models, _NoEventGather(DelayedSimComm(DEV, world=2, delay_us=50)), rings[2], B, d, capture=True)
    _run_es(bad)
    assert not _same([bad_es.engine], [ref_es.engine]), "a missing wait on the batch gather went unnoticed"
