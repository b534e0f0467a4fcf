"""Every ``world > 1`` branch of the graphed multi-GPU steps (``parallel/graphed.py``), executed.

The graphed data-parallel / ZeRO-1 / ensemble-sharded classes are what ``bench.py`` and
``EnsembleTrainer(parallel='dp'|'zero1')`` run at N > 1.  RCCL refuses two ranks on one GPU, so here
2 and 4 gloo ranks share ``cuda:0`` and talk through ``HostComm`` (``parallel/host_comm.py``: the
RcclComm interface, host-staged, so the classes run their step sequence uncaptured).  Each run is
checked against single-process training of the same models on the same global batches
(``ring.graph_source(N B)``: the rank shards concatenate to the single run's batch), replicas are
checked bit-identical, and a line trace of ``graphed.py`` proves the multi-rank branches ran.
Reference: ``experiments/huge_batch_size.py:259-345`` (DDP), ``cluster_runs.py:100-157``.
"""

import ast
import os
import socket
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

D, N_DICT, B = 256, 512, 256
GROUPS = (3, 2, 3)
L1S = (1e-4, 3e-4, 1e-3, 3e-3)
_HITS = {}  # case -> graphed.py lines executed by rank 0


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, mode, grad_dtype, chunks, rows, init, q, sig_name="FunctionalSAE"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from sparse_coding__amd.data.ring import DeviceRing
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.engine.graph_plan import count_pattern
    from sparse_coding__amd.models import signatures
    from sparse_coding__amd.parallel import graphed
    from sparse_coding__amd.parallel.data_parallel import split_models
    from sparse_coding__amd.parallel.dist import DistInfo
    from sparse_coding__amd.parallel.host_comm import HostComm

    FunctionalSAE = getattr(signatures, sig_name)
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda:0")
        dist.init_process_group("gloo", rank=rank, world_size=world)
        info = DistInfo(rank, world, rank, dev, "gloo")
        hits = set()
        target = os.path.abspath(graphed.__file__)

        def tracer(frame, event, arg):
            if frame.f_code.co_filename == target:
                if event == "line":
                    hits.add(frame.f_lineno)
                return tracer
            return None

        ring = DeviceRing(rows.shape[0], D, device=dev, seed=7)
        ring.push(rows.to(dev))
        models = [({k: v.to(dev) for k, v in p.items()}, {k: (v.to(dev) if torch.is_tensor(v) else v)
                                                           for k, v in b.items()}) for p, b in init]
        comm = HostComm(info)
        sys.settrace(tracer)
        if mode == "es":
            from sparse_coding__amd.parallel.ensemble_shard import EnsembleSharded

            es = EnsembleSharded(models, lambda m, bs: FusedSAEEnsemble(m, FunctionalSAE, lr=1e-3, batch_size=bs,
                                                                         device=dev, wgrad_split=1),
                                 info, batch_per_rank=B, d=D)
            runner = graphed.GraphedEnsembleSharded(es, comm, ring.graph_source(B, rank, world))
            assert not runner.capture
            runner.prime([count_pattern(s) for s in set(GROUPS)])
            for s in GROUPS:
                runner.run(s, count_pattern(s))
            torch.cuda.synchronize()
            sys.settrace(None)
            params = {k: v.cpu().numpy() for k, v in es.gather_params().items()}
            e = es.engine
            extra = {"out": e.out.cpu().numpy(), "counts": e.feature_counts.cpu().numpy(),
                     "lo": es.lo, "hi": es.hi, "step": int(e.step_dev.item())}
        else:
            engines = [FusedSAEEnsemble(m, FunctionalSAE, lr=1e-3, batch_size=B, device=dev)
                       for m in split_models(models, chunks)]
            gdp = graphed.GraphedDataParallel(engines, info, comm, ring.graph_source(B, rank, world), mode=mode,
                                              grad_dtype=grad_dtype)
            assert not gdp.capture
            gdp.prime([count_pattern(s) for s in set(GROUPS)])
            for s in GROUPS:
                gdp.run(s, count_pattern(s))
            torch.cuda.synchronize()
            gdp.gather_masters()
            sys.settrace(None)
            params = {k: torch.cat([e.params[k] for e in engines]).cpu().numpy() for k in engines[0].params}
            extra = {"step": int(engines[0].step_dev.item()), "wsplit": [e.wsplit for e in engines]}
        extra["calls"] = dict(comm.calls)
        q.put((rank, params, extra, sorted(hits)))
        dist.destroy_process_group()
    except Exception as exc:  # surface the failure in the parent instead of a queue timeout
        import traceback

        q.put((rank, None, {"error": repr(exc), "tb": traceback.format_exc()}, []))
        raise


MASKED_SIZES = (128, 256, 384, 512)  # live sizes of the masked ensemble (stacked to N_DICT)


def _setup(sig_name="FunctionalSAE"):
    from sparse_coding__amd.models import signatures

    torch.manual_seed(41)
    sig = getattr(signatures, sig_name)
    if "Masked" in sig_name:
        init = [sig.init(D, sz, N_DICT, l1) for sz, l1 in zip(MASKED_SIZES, L1S)]
    else:
        init = [sig.init(D, N_DICT, l1) for l1 in L1S]
    feats = torch.nn.functional.normalize(torch.randn(2048, D), dim=-1)
    rows = ((torch.relu(torch.randn(B * 64, 2048) - 2.0) @ feats) * 1.5).to(torch.bfloat16)
    return init, rows


def _single(init, rows, world, sig_name="FunctionalSAE"):
    """Single-process training of all models on the global batches (N B rows per step)."""
    from sparse_coding__amd.data.ring import DeviceRing
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.engine.graph_plan import count_pattern
    from sparse_coding__amd.models import signatures

    FunctionalSAE = getattr(signatures, sig_name)

    dev = torch.device("cuda:0")
    ring = DeviceRing(rows.shape[0], D, device=dev, seed=7)
    ring.push(rows.to(dev))
    models = [({k: v.to(dev) for k, v in p.items()}, {k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in b.items()})
              for p, b in init]
    e = FusedSAEEnsemble(models, FunctionalSAE, lr=1e-3, batch_size=world * B, device=dev, wgrad_split=1)
    e.enable_graph().attach_source(ring.graph_source(world * B))
    for s in GROUPS:
        e.step_source(s, count_pattern(s))
    torch.cuda.synchronize()
    return e


def _launch(world, mode, grad_dtype=torch.float32, chunks=1, sig_name="FunctionalSAE"):
    import torch.multiprocessing as mp

    init, rows = _setup(sig_name)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, grad_dtype, chunks, rows, init, q, sig_name))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        rank, params, extra, hits = q.get(timeout=240)
        assert params is not None, extra.get("tb")
        res[rank] = (params, extra, hits)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return init, rows, res


def _rel_change(got, want, p0):
    return float(np.linalg.norm(got - want) / (np.linalg.norm(want - p0) + 1e-30))


@pytest.mark.parametrize("world,mode,gdt,chunks", [
    (2, "dp", "fp32", 2), (2, "zero1", "fp32", 1), (2, "zero1", "bf16", 2), (4, "dp", "fp32", 1),
    (4, "zero1", "bf16", 1)])
def test_graphed_data_parallel_multirank(world, mode, gdt, chunks):
    """DP / ZeRO-1 (fp32 reduce-scatter, bf16 all-to-all + owner sums) over N gloo ranks: replicas
    identical after the master gather, and equal to single-process global-batch training."""
    grad_dtype = torch.bfloat16 if gdt == "bf16" else torch.float32
    init, rows, res = _launch(world, mode, grad_dtype, chunks)
    ref = _single(init, rows, world)
    p0s = {k: np.stack([p[k].numpy() for p, _ in init]) for k in res[0][0]}
    for r in range(1, world):
        for k in res[0][0]:
            np.testing.assert_array_equal(res[0][0][k], res[r][0][k], err_msg=f"rank {r} {k}")
    tol = 5e-2 if gdt == "bf16" else 2e-2
    for k, got in res[0][0].items():
        rel = _rel_change(got, ref.params[k].cpu().numpy(), p0s[k])
        assert rel < tol, (k, rel)
    extra = res[0][1]
    assert extra["step"] == sum(GROUPS) and all(w == 1 for w in extra["wsplit"])
    calls = extra["calls"]
    if mode == "dp":
        assert calls.get("all_reduce", 0) >= sum(GROUPS) * chunks
    else:
        assert calls.get("all_to_all" if gdt == "bf16" else "reduce_scatter", 0) >= sum(GROUPS)
        assert calls.get("all_gather", 0) >= sum(GROUPS)
    _HITS[(world, mode, gdt, chunks)] = set(res[0][2])


@pytest.mark.parametrize("world", [2, 4])
def test_graphed_ensemble_sharded_multirank(world):
    """Ensemble sharding over N gloo ranks: in-place all-gathers of the other ranks' slots, each rank's
    models trained on the global batch == the single-process run's models (exact batches, same
    kernels: losses and feature counts match)."""
    init, rows, res = _launch(world, "es")
    ref = _single(init, rows, world)
    p0s = {k: np.stack([p[k].numpy() for p, _ in init]) for k in res[0][0]}
    for r in range(1, world):
        for k in res[0][0]:
            np.testing.assert_array_equal(res[0][0][k], res[r][0][k])
    for k, got in res[0][0].items():
        rel = _rel_change(got, ref.params[k].cpu().numpy(), p0s[k])
        assert rel < 1e-2, (k, rel)
    for r in range(world):
        ex = res[r][1]
        lo, hi = ex["lo"], ex["hi"]
        np.testing.assert_allclose(ex["out"][:, :3], ref.out[lo:hi, :3].cpu().numpy(), rtol=2e-3, atol=1e-6)
        dc = np.abs(ex["counts"] - ref.feature_counts[lo:hi].cpu().numpy())
        assert dc.max() <= 2 and (dc > 0).mean() < 0.01
        assert ex["step"] == sum(GROUPS)
    _HITS[(world, "es")] = set(res[0][2])


@pytest.mark.parametrize("mode,chunks", [("dp", 2), ("zero1", 1)])
def test_graphed_data_parallel_masked_multirank(mode, chunks):
    """A masked ensemble (live sizes 128..512 stacked to 512) data-parallel over 2 gloo ranks: replicas
    identical, equal to single-process global-batch training of the masked models, dead rows unmoved."""
    world = 2
    init, rows, res = _launch(world, mode, torch.float32, chunks, sig_name="FunctionalMaskedSAE")
    ref = _single(init, rows, world, sig_name="FunctionalMaskedSAE")
    assert ref.nactive is not None
    p0s = {k: np.stack([p[k].numpy() for p, _ in init]) for k in res[0][0]}
    for k in res[0][0]:
        np.testing.assert_array_equal(res[0][0][k], res[1][0][k], err_msg=k)
    for k, got in res[0][0].items():
        rel = _rel_change(got, ref.params[k].cpu().numpy(), p0s[k])
        assert rel < 2e-2, (k, rel)
        for g, sz in enumerate(MASKED_SIZES):
            np.testing.assert_array_equal(got[g, sz:], p0s[k][g, sz:], err_msg=f"{k} model {g} dead rows")
    assert res[0][1]["step"] == sum(GROUPS)


def _multirank_lines():
    """Line numbers of graphed.py that only a world > 1 run executes: the first statement of every
    ``if`` whose test is a multi-rank condition (world > 1 / world_size > 1 / lowp), the else of
    ``world == 1`` tests, and the statement after an early return on ``world_size <= 1``."""
    from sparse_coding__amd.parallel import graphed

    tree = ast.parse(open(graphed.__file__).read())
    need = {}
    for node in ast.walk(tree):
        for body_name in ("body", "orelse"):
            stmts = getattr(node, body_name, None)
            if not isinstance(stmts, list):
                continue
            for i, st in enumerate(stmts):
                if not isinstance(st, ast.If):
                    continue
                src = ast.unparse(st.test)
                if "world > 1" in src or "world_size > 1" in src or src.endswith("lowp"):
                    need[st.body[0].lineno] = src
                elif "world == 1" in src and st.orelse:
                    need[st.orelse[0].lineno] = "not " + src
                elif "world_size <= 1" in src and i + 1 < len(stmts):
                    need[stmts[i + 1].lineno] = "not " + src
    return need


def test_every_multirank_branch_executed():
    """Union of the runs above: every multi-rank branch of parallel/graphed.py was executed."""
    if len(_HITS) < 7:
        pytest.skip("needs the multi-rank cases of this module in the same session")
    hit = set().union(*_HITS.values())
    need = _multirank_lines()
    assert len(need) >= 6, need
    missing = {ln: why for ln, why in need.items() if ln not in hit}
    assert not missing, missing
