"""Headline benchmark: activations/sec of a Pythia-70m residual-stream SAE ensemble.

BASELINE.json config 2/3: an 8-way L1 sweep (l1 = logspace(-4, -2, 8)) of untied
SAEs on d_model = 512 activations with dict_ratio 4 (n = 2048), bf16 MFMA compute
with fp32 master weights and fp32 Adam, trained on synthetic Pythia-70m-shaped
activations (sparse mixture of 4096 unit-norm features, held in an HBM ring
buffer; no network, so no real harvest).  Every timed step does the full work:
device-side random batch gather, encoder/decoder forward, backward, Adam on all
8 models (one HIP graph per step on one GPU).

N > 1 GPUs (weak scaling: 2048 rows per GPU per step), ``--parallelism``:
  es  (default) ensemble-axis sharding: rank r owns models [r G/N, (r+1) G/N) and trains
      them on the all-gathered global batch -- per model the same update as data parallel
      on the global batch, but 2 MB of batch cross xGMI per step instead of 67 MB of
      gradients;
  dp  data parallel: every rank holds all 8 models, gradients are all-reduced (RCCL over
      xGMI) in model chunks overlapped with the next chunk's compute (BASELINE config 3's
      mechanism); each chunk's kernels replay from HIP graphs.
  zero1  data parallel with ZeRO-1: reduce-scatter of the gradients onto row owners, Adam on
      the owned rows only, all-gather of the bf16 shadows (parallel/zero.py).
The run times the other strategy too (untimed for the headline) and reports it under
``alt_parallelism`` in the JSON line.

Run:  python bench.py [--gpus N --steps K --warmup W]
      torchrun --nproc-per-node N bench.py --gpus N ...
Prints one JSON line (rank 0).
"""

from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

# the reference's untied 8-model d=512 n=2048 step (its own math,
# vmap(grad)+Adam) -- the only measured throughput for this exact config (no GPU number
# is published, BASELINE.json "published": {}).
BASELINE_ACT_PER_S = 1.86e3
# This repo's PyTorch-eager engine (FunctionalEnsemble: torch.func vmap(grad(loss)) + vmapped
# Adam, fp32, the reference's algorithm) on ONE MI355X at the same config, measured with
# ``bench.py --engine eager`` (profiles/bench_eager_r2.json: 2.63 ms/step).
EAGER_SAME_BOX_ACT_PER_S = 779054.6
# single-GPU step and per-rank ensemble-sharded steps measured on one MI355X (inputs of the
# comm model's prediction, parallel/comm_model.py; round 4: profiles/r4/final_defaults/long_*.json,
# profiles/r4/es_projection/es_projection_r4.jsonl -- G/N models on N B rows, single-step graphs)
T1_MS = 0.300
ES_MS = {2: 0.2657, 4: 0.246, 8: 0.2374}
METRIC = "activations/sec (ensemble train) + FVU@L0, Pythia-70m resid SAE at 1/2/4/8 GPU"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=2048, help="rows per GPU per step")
    ap.add_argument("--d", type=int, default=512)
    ap.add_argument("--ratio", type=int, default=4)
    ap.add_argument("--models", type=int, default=8)
    ap.add_argument("--kind", choices=["untied", "tied"], default="untied")
    ap.add_argument("--engine", choices=["fused", "eager"], default="fused")
    ap.add_argument("--ring-rows", type=int, default=1 << 21)
    ap.add_argument("--eval-rows", type=int, default=16384)
    ap.add_argument("--act-norm", type=float, default=9.0,
                    help="mean L2 norm the synthetic rows are scaled to.  Calibrated on the reference's "
                         "shipped Pythia-70m layer-2 TiedSAE (l1=1e-3: L0~77, unit-norm atoms, bias ~-0.85 "
                         "=> |x|^2 ~ 77 codes of O(1)), so the reference's L1 range logspace(-4,-2) spans "
                         "dense to very sparse codes as it does on the real activations")
    ap.add_argument("--quality-steps", type=int, default=3000,
                    help="after the timed region, keep training (untimed) until this many steps in total "
                         "before the FVU@L0 evaluation (the timed K steps alone are far from converged)")
    ap.add_argument("--grad-dtype", choices=["fp32", "bf16"], default=None,
                    help="gradient transport of the data-parallel modes (default: dp fp32 all-reduce; zero1 bf16 "
                         "all-to-all with fp32 accumulation on the row owner, parallel/zero.py)")
    ap.add_argument("--parallelism", choices=["auto", "es", "dp", "zero1"], default="auto",
                    help="N>1: 'es' = ensemble-axis sharding (each GPU owns models/N models and trains "
                         "them on the all-gathered global batch: identical updates to data parallel on the "
                         "global batch, but only the 2 MB batch crosses xGMI instead of 67 MB of gradients); "
                         "'dp' = data parallel with chunk-pipelined RCCL gradient all-reduce; 'zero1' = data "
                         "parallel with reduce-scatter, row-sharded Adam and a bf16 shadow all-gather; "
                         "auto = the mode parallel/comm_model.py predicts fastest at this N")
    ap.add_argument("--dp-chunks", type=int, default=None,
                    help="dp / zero1: split the ensemble into this many model chunks whose gradient all-reduce "
                         "overlaps the next chunk's compute (1 = one reduction per step; default 2, or 1 on "
                         "one rank, where there is no communication to hide)")
    ap.add_argument("--dist-backend", choices=["auto", "nccl", "gloo"], default="auto",
                    help="auto = RCCL ('nccl') on GPUs; gloo only for rehearsals")
    ap.add_argument("--shared-gpu", action="store_true",
                    help="rehearsal: every rank on cuda:0 (with --dist-backend gloo on a 1-GPU box)")
    ap.add_argument("--force-dist", action="store_true",
                    help="create the process group even at N=1 and run the N>1 code path (rehearses the "
                         "sharded step with real RCCL collectives on a one-GPU box)")
    ap.add_argument("--no-eval", action="store_true")
    ap.add_argument("--no-comm-calibration", action="store_true",
                    help="N > 1: skip timing the node's collectives before choosing the mode (link model only)")
    ap.add_argument("--wgrad-dtype", choices=["fp32", "bf16"], default="fp32",
                    help="single GPU: storage of the weight gradients between the wgrad GEMM and Adam (the "
                         "moments, masters and the update stay fp32)")
    ap.add_argument("--graph-group", type=int, default=None,
                    help="steps per graph replay (default: engine/graph_plan.tile's choice, <= 10)")
    ap.add_argument("--settle-mode", choices=["gemm", "step"], default="step",
                    help="settle load: 'gemm' = the grouped GEMM on scratch operands; 'step' = the same fused "
                         "step on a scratch ensemble of the benchmark's shapes (discarded, shares no state)")
    ap.add_argument("--settle-ms", type=float, default=150.0,
                    help="untimed non-training GPU load before the warmup so the timed steps run at the "
                         "steady-state clock (settle_clocks; reported as 'settle' in the JSON; 0 = off)")
    ap.add_argument("--compare-parallelism", type=int, default=1,
                    help="N>1: after the headline run, also time the other strategy (es <-> dp) and report it "
                         "under alt_parallelism")
    ap.add_argument("--no-graph", action="store_true", help="launch kernels eagerly instead of HIP graphs")
    ap.add_argument("--dist-graph", "--dp-graph", dest="dist_graph", type=int, default=1,
                    help="N>1 / --force-dist: 1 = multi-step HIP graphs with the RCCL collectives captured inside "
                         "them (parallel/graphed.py, native communicator on its own stream: es all-gathers, dp "
                         "all-reduce, zero1 reduce-scatter / all-gather); 0 = host-issued collectives through "
                         "ProcessGroupNCCL between graph replays (parallel/ensemble_shard.py, data_parallel.py, zero.py)")
    ap.add_argument("--fallback-reason", default=None,
                    help="(set by launch_ranks when it relaunches after a watchdog exit) why this run uses "
                         "host-issued collectives; reported as collectives.fallback")
    ap.add_argument("--watchdog-scale", type=float, default=1.0,
                    help="N > 1: multiplies every per-phase watchdog limit (WATCHDOG_S); 0 = no watchdog")
    return ap.parse_args(argv)


def build_ring(args, device):
    from sparse_coding__amd.data.ring import DeviceRing
    from sparse_coding__amd.data.synthetic import RandomDatasetGenerator

    gen = RandomDatasetGenerator(activation_dim=args.d, n_ground_truth_components=8 * args.d,
                                 batch_size=65536, feature_num_nonzero=32, feature_prob_decay=0.999,
                                 correlated=False, device=device, seed=1234)
    probe = gen.send(None)
    scale = args.act_norm / float(probe.norm(dim=-1).mean()) if args.act_norm > 0 else 1.0
    ring = DeviceRing(args.ring_rows, args.d, device=device, seed=4321)
    ring.fill(lambda: gen.send(None) * scale)
    held_out = gen.send(None)[: args.eval_rows] * scale
    return ring, held_out


def fvu_l0(dicts, x):
    from sparse_coding__amd.eval.metrics import fraction_variance_unexplained, mean_l0

    return [(float(mean_l0(ld, x)), float(fraction_variance_unexplained(ld, x))) for ld in dicts]


# single-GPU fused step: at most this many optimizer steps per HIP graph replay (each replay
# boundary costs an ~9 us idle gap on MI355X); engine/graph_plan.py picks the tiling with the fewest
# timed replays -- the warmup replays the timed graphs first only when it is long enough
# ("graph_replays.warm_covered" in the JSON; every graph is captured and uploaded before the warmup)
GRAPH_STEPS = 10


class Runner:
    """One training configuration.

    ``setup(tiling)``: capture (and upload) every graph the run will replay -- before warmup;
    ``run(groups)``: one full optimizer step per entry of ``sum(groups)``, replayed as one graph per
    group where the runner has graphs; ``finish()``: complete cross-step work in flight;
    ``dicts()``: LearnedDicts; ``close()``."""

    def __init__(self, step, dicts, finish=None, close=None, run=None, setup=None):
        self.step, self.dicts = step, dicts
        self.path, self.comm, self.consistency = "single", None, None
        self.fallback = None  # why the in-graph path was abandoned for host-issued collectives
        self.finish = finish or (lambda: None)
        self.close = close or (lambda: None)
        self._run = run
        self.setup = setup or (lambda tiling: None)

    def run(self, groups):
        if self._run is not None:
            return self._run(groups)
        for _ in range(sum(groups)):
            self.step()


def _graph_comm(info, args):
    """The communicator the in-graph (graphed) multi-GPU paths run on, and what it is:
    ``("rccl", RcclComm)`` -- the native RCCL communicator whose collectives are captured in the step
    graphs; ``("gloo", HostComm)`` -- gloo rehearsals (e.g. ranks sharing one GPU): the same graphed
    step sequence, run uncaptured with host-staged collectives; ``(reason, None)`` -- no native
    communicator here: the runner uses host-issued ProcessGroupNCCL collectives."""
    if info.backend == "gloo":
        from sparse_coding__amd.parallel.host_comm import HostComm

        return "gloo", HostComm(info)
    from sparse_coding__amd.parallel.rccl import RcclComm

    try:
        return "rccl", RcclComm(info)
    except Exception as exc:  # e.g. no librccl symbols / ncclCommInitRank error
        print(f"[bench] native RCCL communicator unavailable ({exc!r}); host-issued collectives", file=sys.stderr)
        return f"native RCCL communicator unavailable: {exc!r}", None


PATH_NAMES = {
    "single": "none (one GPU, no collectives)",
    "rccl": "in-graph RCCL (native communicator, collectives captured in the multi-step HIP graphs)",
    "gloo": "graphed step sequence uncaptured, gloo host-staged collectives (rehearsal)",
    "host": "host-issued ProcessGroup collectives between HIP graph replays",
    "eager": "eager engine, host-issued ProcessGroup collectives",
}


def make_runner(par, args, info, sig, models, ring, device, grad_dtype, dist_graph=None):
    """The runner of one training configuration.  ``runner.path`` names the collective path
    (PATH_NAMES); ``runner.comm`` is the graphed paths' communicator; ``runner.consistency()``
    (collective, every rank) checks the ranks agree after the run."""
    B = args.batch
    distributed = info.world_size > 1 or args.force_dist
    dist_graph = args.dist_graph if dist_graph is None else dist_graph
    if args.engine == "fused" and par == "es":
        from sparse_coding__amd.engine.fused import FusedSAEEnsemble
        from sparse_coding__amd.parallel.ensemble_shard import EnsembleSharded

        from sparse_coding__amd.engine.graph_plan import count_pattern

        es = EnsembleSharded(models, lambda m, bs: FusedSAEEnsemble(m, sig, lr=1e-3, batch_size=bs, device=device),
                             info, batch_per_rank=B, d=args.d)
        metas = [b for _, b in models]

        def sample(out):
            return ring.sample_shard(B, info.rank, info.world_size, out=out)

        def dicts():
            return es.to_learned_dicts(metas, sig, device)

        if args.no_graph:
            r = Runner(lambda: es.step_sampled(sample), dicts, close=es.flush)
            r.path, r.consistency = "host", lambda: _batch_spread(es.gbuf, info)
            return r
        kind, comm = _graph_comm(info, args) if dist_graph and distributed else ("host", None)
        if comm is not None:
            # the group's batch fetch and in-place all-gathers captured in its graph (parallel/graphed.py)
            from sparse_coding__amd.parallel.graphed import GraphedEnsembleSharded

            ges = GraphedEnsembleSharded(es, comm, ring.graph_source(B, info.rank, info.world_size))

            def run_g(groups):
                for s in groups:
                    ges.run(s, count_pattern(s, GRAPH_STEPS))

            r = Runner(lambda: run_g([1]), dicts, close=comm.close, run=run_g,
                       setup=lambda tiling: ges.prime([count_pattern(s, GRAPH_STEPS) for s in tiling.sizes]))
            r.path, r.comm = kind, comm
            r.consistency = lambda: _batch_spread([ges._glob], info)
            return r

        def sample_steps(out, s):  # this rank's rows of the next s steps, one gather kernel
            return ring.sample_shard_steps(B, info.rank, info.world_size, s, out)

        def pattern(s):
            return count_pattern(s, GRAPH_STEPS)

        # multi-step groups: per group one local-row gather, s batch all-gathers (RCCL stream, issued
        # under the previous group's replay) and ONE HIP graph replay of the s steps
        r = Runner(lambda: es.run_groups([1], sample_steps, pattern), dicts, close=es.flush,
                   run=lambda groups: es.run_groups(groups, sample_steps, pattern),
                   setup=lambda tiling: (ring.ensure_permutation(), es.prime_groups(tiling.sizes, pattern)))
        r.path = "host"
        r.consistency = lambda: _batch_spread(getattr(es, "_gglob", es.gbuf), info)
        return r
    kind, comm = (_graph_comm(info, args) if args.engine == "fused" and distributed and not args.no_graph and dist_graph
                  else ("host", None))
    if comm is not None:
        # data parallel / ZeRO-1 with the collectives INSIDE multi-step HIP graphs (native RCCL
        # communicator on its own stream, parallel/rccl.py + parallel/graphed.py)
        from sparse_coding__amd.engine.fused import FusedSAEEnsemble
        from sparse_coding__amd.engine.graph_plan import count_pattern
        from sparse_coding__amd.parallel.data_parallel import split_models
        from sparse_coding__amd.parallel.graphed import GraphedDataParallel

        # flat fp32 gradients (no split-K slabs): the reductions read the engines' grad_all
        engines = [FusedSAEEnsemble(m, sig, lr=1e-3, batch_size=B, device=device, wgrad_split=1)
                   for m in split_models(models, args.dp_chunks)]
        gdp = GraphedDataParallel(engines, info, comm, ring.graph_source(B, info.rank, info.world_size), mode=par,
                                  grad_dtype=grad_dtype)

        def run(groups):
            for s in groups:
                gdp.run(s, count_pattern(s, GRAPH_STEPS))

        def masters():
            gdp.gather_masters()
            return [t for e in engines for k in sorted(e.params) for t in (e.params[k],)]

        r = Runner(lambda: run([1]), lambda: gdp.to_learned_dicts(device), close=comm.close, run=run,
                   setup=lambda tiling: gdp.prime([count_pattern(s, GRAPH_STEPS) for s in tiling.sizes]))
        r.path, r.comm = kind, comm
        r.consistency = lambda: _replica_delta(masters(), info)
        return r
    if args.engine == "fused" and distributed:
        from sparse_coding__amd.engine.fused import FusedSAEEnsemble
        from sparse_coding__amd.parallel.data_parallel import ChunkedDataParallel, FusedChunk, split_models
        from sparse_coding__amd.parallel.zero import ZeroFusedChunk

        engines = [FusedSAEEnsemble(m, sig, lr=1e-3, batch_size=B, device=device, wgrad_split=1)
                   for m in split_models(models, args.dp_chunks)]
        xbuf = torch.empty(B, args.d, device=device, dtype=torch.bfloat16)
        graph = not args.no_graph  # each chunk's compute and update replay from HIP graphs
        if par == "zero1":
            chunks = [ZeroFusedChunk(e, info, grad_dtype, graph=graph, x_static=xbuf) for e in engines]
        else:
            chunks = [FusedChunk(e, graph=graph, x_static=xbuf) for e in engines]
        # cross-step: the last chunk's collectives overlap the next step's first (encoder) GEMMs
        trainer = ChunkedDataParallel(chunks, info, grad_dtype, cross_step=True)

        def gather():
            trainer.flush()
            for c in chunks:  # ZeRO-1: every rank gathers the current masters before exporting
                if hasattr(c, "gather_masters"):
                    c.gather_masters()

        def dicts():
            gather()
            return [ld for e in engines for ld in e.to_learned_dicts(device)]

        def masters():
            gather()
            return [t for e in engines for k in sorted(e.params) for t in (e.params[k],)]

        r = Runner(lambda: trainer.step_batch(ring.sample_shard(B, info.rank, info.world_size, out=xbuf)),
                   dicts, finish=trainer.flush, close=trainer.flush)
        r.path, r.consistency = "host", lambda: _replica_delta(masters(), info)
        return r
    if args.engine == "fused":
        from sparse_coding__amd.engine.fused import FusedSAEEnsemble

        from sparse_coding__amd.engine.graph_plan import count_pattern

        eng = FusedSAEEnsemble(models, sig, lr=1e-3, batch_size=B, device=device, grad_dtype=args.wgrad_dtype)
        if args.no_graph:
            def step():
                ring.sample_shard(B, 0, 1, out=eng.x_static)
                eng.step_batch(eng.x_static)

            return Runner(step, lambda: eng.to_learned_dicts(device))
        # every step (ring batch gather included) runs from HIP graphs of up to GRAPH_STEPS steps;
        # feature counts are sampled on the first step of each replay (every <= 8 steps)
        eng.enable_graph().attach_source(ring.graph_source(B))

        def run(groups):
            for s in groups:
                eng.step_source(s, count_pattern(s, GRAPH_STEPS))

        def setup(tiling):
            eng.prime_source(patterns=[count_pattern(s, GRAPH_STEPS) for s in tiling.sizes])

        return Runner(lambda: run([1]), lambda: eng.to_learned_dicts(device), run=run, setup=setup)
    from sparse_coding__amd.engine.ensemble import FunctionalEnsemble
    from sparse_coding__amd.engine.optim import adam
    from sparse_coding__amd.parallel.data_parallel import DataParallelEnsemble

    ens = FunctionalEnsemble(models, sig, adam, {"lr": 1e-3}, device=device)
    trainer = DataParallelEnsemble(ens, info)
    r = Runner(lambda: trainer.step_batch(ring.sample_shard(B, info.rank, info.world_size).float()),
               lambda: ens.to_learned_dicts(device))
    r.path = "eager" if distributed else "single"
    r.consistency = lambda: _replica_delta([ens.params[k] for k in sorted(ens.params)], info)
    return r


def _replica_delta(tensors, info):
    """Data parallel: max |p - p_rank0| over every master and rank (0.0 = replicas identical).
    Collective."""
    import torch.distributed as tdist

    worst = 0.0
    for t in tensors:
        mine = t.detach().contiguous()
        if info.backend == "gloo":
            mine = mine.cpu()
        ref = mine.clone()
        tdist.broadcast(ref, src=0)
        worst = max(worst, float((mine.float() - ref.float()).abs().max()))
    from sparse_coding__amd.parallel.dist import all_reduce_max

    return {"what": "max |master - rank 0's master| over all parameters and ranks (after the ZeRO-1 gather)",
            "max_abs_delta": all_reduce_max(worst, info)}


def _batch_spread(bufs, info):
    """Ensemble sharding: every rank must have trained on the same global batches.  Checksums of the
    gathered global-batch buffers (sum and an index-weighted sum in fp64) compared across ranks."""
    import torch.distributed as tdist

    sums = []
    for b in bufs:
        if b is None:
            continue
        x = b.detach().double().reshape(-1)
        w = torch.arange(x.numel(), device=x.device, dtype=torch.float64).remainder_(9973).add_(1)
        sums += [float(x.sum()), float((x * w).sum())]
    everyone = [None] * info.world_size
    tdist.all_gather_object(everyone, sums)
    spread = max((abs(a - b) for other in everyone for a, b in zip(other, everyone[0])), default=0.0)
    return {"what": "spread over ranks of fp64 checksums of the last gathered global batches (0.0 = identical)",
            "checksums_rank0": everyone[0], "max_abs_spread": spread}


def comm_bytes(mode, args, world):
    """Per-GPU bytes sent per step by the data-parallel modes at this config (parallel/zero.py):
    dp all-reduces the weight + bias gradients, zero1 reduce-scatters them and all-gathers the
    bf16 shadows, es all-gathers the batch."""
    from sparse_coding__amd.parallel.zero import comm_bytes_per_step

    n = args.d * args.ratio
    params = args.models * (2 * n * args.d + n)
    gbytes = 2 if args.grad_dtype == "bf16" else 4
    return comm_bytes_per_step(mode, world, params * gbytes, shadow_bytes=args.models * 2 * n * args.d * 2,
                               batch_bytes=world * args.batch * args.d * 2)  # gathered global batch


def timed(runner, groups, info, B):
    """Exactly ``sum(groups)`` steps between barrier + synchronize on both sides; max over ranks."""
    from sparse_coding__amd.parallel.dist import all_reduce_max, barrier

    steps = sum(groups)
    # (diagnostic only: device events on the current stream around the same region -- what the GPU
    # saw from the first timed launch to the last, without the host's first-launch latency)
    cuda = torch.cuda.is_available()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)] if cuda else None
    barrier(info)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if ev:
        ev[0].record()
    runner.run(groups)
    runner.finish()  # work the last timed step still has in flight (cross-step pipelining)
    if ev:
        ev[1].record()
    torch.cuda.synchronize()
    barrier(info)
    elapsed = all_reduce_max(time.perf_counter() - t0, info)
    runner.gpu_event_ms = (all_reduce_max(ev[0].elapsed_time(ev[1]) / 1e3, info) * 1e3 / steps) if ev else None
    return 1e3 * elapsed / steps, B * info.world_size * steps / elapsed


def settle_step(device, ms: float, args):
    """Untimed settle load with the step's own kernel mix: a SCRATCH ensemble of the benchmark's
    shapes (fresh random weights, its own buffers and graph, a fixed random batch) replays its
    training step for ``ms`` milliseconds and is then discarded.  Nothing of the measured models is
    read or written."""
    if ms <= 0:
        return None
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.models.signatures import FunctionalSAE, FunctionalTiedSAE

    sig = FunctionalSAE if args.kind == "untied" else FunctionalTiedSAE
    n = args.d * args.ratio
    gen = torch.Generator(device=device).manual_seed(11)
    scratch = [sig.init(args.d, n, 1e-3, device=device) for _ in range(args.models)]
    eng = FusedSAEEnsemble(scratch, sig, lr=1e-3, batch_size=args.batch, device=device).enable_graph()
    eng.x_static.copy_(torch.randn(args.batch, args.d, device=device, generator=gen).to(torch.bfloat16))
    eng.step_batch(eng.x_static)  # capture
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    steps = 0
    while 1e3 * (time.perf_counter() - t0) < ms:
        for _ in range(16):
            eng.step_batch(eng.x_static)
        steps += 16
        torch.cuda.synchronize()
    out = {"what": "the fused training step on a scratch ensemble of the same shapes (discarded; no state "
                   "shared with the measured models)", "ms": round(1e3 * (time.perf_counter() - t0), 1),
           "steps": steps}
    del eng, scratch
    return out


def time_layout(device, sig, args, models: int, rows: int, steps: int = 12, warm: int = 4) -> float:
    """ms per fused training step of ``models`` SAEs of the benchmark's shape on ``rows`` rows (a
    scratch ensemble, single-step graphs on a fixed random batch; nothing of the measured models)."""
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble

    n = args.d * args.ratio
    gen = torch.Generator(device=device).manual_seed(13)
    scratch = [sig.init(args.d, n, 1e-3, device=device) for _ in range(models)]
    eng = FusedSAEEnsemble(scratch, sig, lr=1e-3, batch_size=rows, device=device).enable_graph()
    eng.x_static.copy_(torch.randn(rows, args.d, device=device, generator=gen).to(torch.bfloat16))
    for _ in range(warm):
        eng.step_batch(eng.x_static)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.step_batch(eng.x_static)
    torch.cuda.synchronize()
    ms = 1e3 * (time.perf_counter() - t0) / steps
    del eng, scratch
    return ms


def calibrate_compute(info, args, sig, shape):
    """N > 1 (collective): time the per-rank compute layout of each candidate mode ON THIS NODE -- all G
    models on B rows (dp / zero1) and G/N models on N B rows (es) -- max over ranks, and feed them to
    the comm model (``StepShape.use_measured_compute``) before ``best_mode``.  Untimed for the headline;
    reported as ``compute_calibration`` next to ``predicted_ms_per_step``."""
    from sparse_coding__amd.parallel.dist import all_reduce_max

    world = info.world_size
    if world <= 1 or args.engine != "fused" or info.device.type != "cuda":
        return None
    t1 = all_reduce_max(time_layout(info.device, sig, args, args.models, args.batch), info)
    es = None
    if args.models % world == 0:
        es = all_reduce_max(time_layout(info.device, sig, args, args.models // world, args.batch * world), info)
    shape.use_measured_compute(world, t1, es)
    return {"what": "fused step of each mode's per-rank layout timed on this node (scratch ensembles, "
                    "single-step graphs, max over ranks) -- the comm model's compute inputs",
            "t1_ms": round(t1, 4), "es_ms": round(es, 4) if es else None,
            "constants_replaced": {"t1_ms": T1_MS, "es_ms": ES_MS.get(world)}}


def settle_clocks(device, ms: float):
    """Untimed, NON-training GPU load before the warmup: the grouped bf16 MFMA GEMM (the step's own
    kernel, plain epilogue) on scratch random operands for ``ms`` milliseconds.  MI355X raises its
    clock over the first ~100 ms of sustained load (profiles/settle_r4.jsonl: a run started from an
    idle GPU takes 351 us per step over its first 20 steps, 328 us by 20 ms, 324-325 us from 100 ms
    on), so a 20-step timed region that starts on a cold GPU measures the ramp, not the step.
    Touches no training state.  Returns what ran (reported in the JSON)."""
    if ms <= 0:
        return None
    from sparse_coding__amd.ops import gemm as gemm_ops

    g = torch.Generator(device=device).manual_seed(7)
    a = torch.randn(2048, 512, device=device, generator=g).to(torch.bfloat16)
    b = torch.randn(8, 2048, 512, device=device, generator=g).to(torch.bfloat16)
    out = torch.empty(8, 2048, 2048, device=device, dtype=torch.bfloat16)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    launches = 0
    while 1e3 * (time.perf_counter() - t0) < ms:
        for _ in range(25):
            gemm_ops.matmul_nt(a, b, out)
        launches += 25
        torch.cuda.synchronize()
    return {"what": "grouped bf16 MFMA GEMM 8 x 2048x2048x512 on scratch buffers (no training state)",
            "ms": round(1e3 * (time.perf_counter() - t0), 1), "launches": launches}


HANG_RC = 5  # a rank's exit code when the watchdog ended a hung phase (launch_ranks relaunches on it)
HANG_DIR_ENV = "SC_BENCH_HANG_DIR"  # where a firing watchdog leaves its marker for launch_ranks


class Watchdog:
    """Bounds every multi-rank phase of the run so the first real N > 1 run cannot end without a
    JSON line (a hang inside a captured RCCL collective blocks ``torch.cuda.synchronize()`` until the
    process-group timeout, and no exception ever reaches ``ready_runner``'s fallback).

    ``arm(phase, seconds)`` starts the clock for a phase, ``disarm()`` stops it.  When a phase
    overruns, the watchdog thread prints the phase and rank, writes a marker ``rank<r>.json`` under
    ``$SC_BENCH_HANG_DIR`` (set by ``launch_ranks``), emits ``pending`` -- a finished result record,
    when the hang happens after the headline was measured (the alt-parallelism run, shutdown) -- and
    ends the process with ``os._exit(HANG_RC)``.  No exec, no retry in this process: a device fault
    or a hung collective leaves the process's HIP state unusable, so ``launch_ranks`` starts FRESH
    ranks with ``--dist-graph 0``.  Reference: ``experiments/huge_batch_size.py:337-363`` (mp.spawn of
    the DDP ranks; no hang handling there)."""

    def __init__(self, info, enabled: bool, scale: float = 1.0):
        import threading

        self.info, self.enabled, self.scale = info, enabled, scale
        self.pending = None  # a finished record rank 0 emits if a later phase hangs
        self._lock = threading.Lock()
        self._phase, self._deadline, self._gen = None, None, 0
        self._wake = threading.Event()
        self.fired = None
        if enabled:
            threading.Thread(target=self._watch, name="bench-watchdog", daemon=True).start()

    def arm(self, phase: str, seconds: float):
        with self._lock:
            self._phase, self._deadline = phase, time.monotonic() + seconds * self.scale
            self._gen += 1
        self._wake.set()

    def disarm(self):
        with self._lock:
            self._phase, self._deadline = None, None
            self._gen += 1
        self._wake.set()

    def _watch(self):
        while True:
            with self._lock:
                phase, deadline, gen = self._phase, self._deadline, self._gen
            self._wake.clear()
            if deadline is None:
                self._wake.wait()
                continue
            left = deadline - time.monotonic()
            if left > 0:
                self._wake.wait(left)
                continue
            with self._lock:
                if gen != self._gen:  # re-armed or disarmed meanwhile
                    continue
            self._fire(phase)
            return

    def fire_now(self, phase: str):
        """End the process now as if ``phase`` had hung (a failure this process cannot recover from)."""
        self._fire(phase)

    def _fire(self, phase: str):
        rank = getattr(self.info, "rank", 0)
        self.fired = phase
        print(f"[bench] watchdog: rank {rank} hung in phase '{phase}'; exiting {HANG_RC}", file=sys.stderr, flush=True)
        where = os.environ.get(HANG_DIR_ENV)
        if where:
            try:
                with open(os.path.join(where, f"rank{rank}.json"), "w") as f:
                    json.dump({"rank": rank, "phase": phase, "emitted": self.pending is not None}, f)
            except OSError:
                pass
        if self.pending is not None and getattr(self.info, "is_main", True):
            rec = dict(self.pending)
            rec.setdefault("watchdog", {"phase": phase, "note": "this phase hung after the headline was "
                                                                 "measured; the record is complete up to it"})
            try:
                _emit(json.dumps(rec))
            except Exception:
                pass
        sys.stderr.flush()
        os._exit(HANG_RC)


# per-phase limits (seconds) of the N > 1 watchdog; every one is far above a healthy run's time
WATCHDOG_S = {"setup": 240.0, "first-replay": 120.0, "timed": 240.0, "eval": 300.0, "checks": 120.0,
              "alt": 400.0, "shutdown": 60.0}


def _agree(err, info):
    """Every rank's error (or None) -> the first one any rank reported (collective; the ranks must
    all take the same path afterwards or the next collective deadlocks)."""
    if info.world_size <= 1:
        return err
    import torch.distributed as tdist

    everyone = [None] * info.world_size
    tdist.all_gather_object(everyone, err)
    return next((f"rank {r}: {e}" for r, e in enumerate(everyone) if e is not None), None)


def ready_runner(par, args, info, sig, models, ring, device, grad_dtype, wd=None, tag=""):
    """``make_runner`` + capture of every graph (+ the first warmup group for the in-graph RCCL path).
    If capturing or first replaying the in-graph collectives RAISES on any rank, every rank drops that
    runner and rebuilds the same configuration (fresh from ``models``) on host-issued collectives
    (``--dist-graph 0``) in this process; the JSON reports it (``collectives.fallback``).  A HANG in
    either phase is the watchdog's (``wd``): the rank exits ``HANG_RC`` and ``launch_ranks`` relaunches
    fresh ranks on host-issued collectives.  Returns (runner, tiling, warmup groups still to run)."""
    from sparse_coding__amd.engine.graph_plan import tile

    wd = wd or Watchdog(info, False)
    tiling = tile(args.steps, args.warmup, args.graph_group or GRAPH_STEPS, exact=bool(args.graph_group))
    warm = list(tiling.warm)
    wd.arm(f"{tag}setup", WATCHDOG_S["setup"])
    runner = make_runner(par, args, info, sig, models, ring, device, grad_dtype)
    if runner.path != "rccl":
        runner.setup(tiling)
        wd.disarm()
        return runner, tiling, warm
    err = None
    try:
        runner.setup(tiling)
    except Exception as exc:
        err = f"capture of the in-graph collectives failed: {exc!r}"
    err = _agree(err, info)
    if err is None and warm:
        wd.arm(f"{tag}first-replay", WATCHDOG_S["first-replay"])
        replay_err = None
        try:
            runner.run(warm[:1])
            runner.finish()
            torch.cuda.synchronize()
        except Exception as exc:
            replay_err = f"first replay of the in-graph collectives failed: {exc!r}"
        if replay_err is not None and wd.enabled:
            # a replay error may be a device fault, which is sticky: this process cannot rebuild on
            # host collectives, fresh ranks can (launch_ranks relaunches on the watchdog's exit code)
            wd.fire_now(f"{tag}first-replay raised: {replay_err}")
        err = _agree(replay_err, info)
        if err is None:
            warm = warm[1:]
    wd.disarm()
    if err is None:
        return runner, tiling, warm
    wd.arm(f"{tag}fallback-setup", WATCHDOG_S["setup"])
    print(f"[bench] {err}; falling back to host-issued collectives (--dist-graph 0)", file=sys.stderr)
    try:
        runner.close()
    except Exception as exc:  # the communicator may be unusable; the fallback does not need it
        print(f"[bench] closing the failed communicator: {exc!r}", file=sys.stderr)
    runner = make_runner(par, args, info, sig, models, ring, device, grad_dtype, dist_graph=0)
    runner.fallback = err
    runner.setup(tiling)
    wd.disarm()
    return runner, tiling, list(tiling.warm)


def warm_and_time(runner, tiling, warm, args, info, B):
    """Graphs are captured (``ready_runner``); settle the clocks (untimed, non-training, reported), run
    the warmup (through the timed region's own graphs when it is long enough: ``tiling.covered``),
    then time exactly ``args.steps`` steps (engine/graph_plan.py)."""
    runner.settle = (settle_step(info.device, args.settle_ms, args) if args.settle_mode == "step"
                     else settle_clocks(info.device, args.settle_ms))
    runner.run(warm)
    runner.finish()  # no warmup work may spill into the timed region
    ms, value = timed(runner, list(tiling.timed), info, B)
    return ms, value


def _in_torchrun() -> bool:
    return "WORLD_SIZE" in os.environ and "RANK" in os.environ


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(gpus: int, argv, script: str | None = None) -> int:
    """``--gpus N > 1`` outside torchrun: start N rank processes (``torch.distributed.run``, one per GPU,
    rendezvous on 127.0.0.1) and forward rank 0's JSON line.  This process does no GPU work (it only
    counted devices, which does not initialise HIP) and exits with the launcher's return code
    (non-zero when any rank failed).  Reference: ``experiments/huge_batch_size.py:358-363``
    (``mp.spawn(..., nprocs=torch.cuda.device_count())``)."""
    import subprocess

    import shutil
    import tempfile

    def once(args_):
        hang_dir = tempfile.mkdtemp(prefix="sc_bench_hang_")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
               script or os.path.abspath(__file__)] + list(args_)
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        env[HANG_DIR_ENV] = hang_dir
        print(f"[bench] launching {gpus} ranks: {' '.join(cmd)}", file=sys.stderr)
        proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
        emitted = 0
        for line in proc.stdout:
            if line.startswith("{") and '"metric"' in line and emitted == 0:
                _emit(line.strip())
                emitted += 1
            else:
                sys.stderr.write(line)
        rc = proc.wait()
        hangs = []
        for name in sorted(os.listdir(hang_dir)):
            try:
                with open(os.path.join(hang_dir, name)) as f:
                    hangs.append(json.load(f))
            except (OSError, ValueError):
                pass
        shutil.rmtree(hang_dir, ignore_errors=True)
        return rc, emitted, hangs

    rc, emitted, hangs = once(argv)
    if hangs and emitted == 0 and not _dist_graph_off(argv):
        # a rank's watchdog ended a hung phase before any result: fresh ranks (the hung processes' HIP
        # state is not reusable) on host-issued collectives, with the reason on record
        phase = hangs[0]["phase"]
        reason = f"in-graph hang: {phase} (rank {hangs[0]['rank']}); relaunched with --dist-graph 0"
        print(f"[bench] {reason}", file=sys.stderr)
        rc, emitted, hangs = once(list(argv) + ["--dist-graph", "0", "--fallback-reason", reason])
    if emitted == 1 and rc != 0 and hangs:
        # the result line is out and a watchdog ended a later phase (shutdown, the alt-parallelism run)
        print(f"[bench] ranks exited {rc} after the result line (watchdog: {hangs})", file=sys.stderr)
        return 0
    if rc == 0 and emitted != 1:
        print(f"[bench] the ranks exited 0 but printed {emitted} result lines", file=sys.stderr)
        return 4
    return rc


def _dist_graph_off(argv) -> bool:
    """True when ``argv`` already asks for host-issued collectives (``--dist-graph 0``)."""
    argv = list(argv)
    for i, a in enumerate(argv):
        if a in ("--dist-graph", "--dp-graph") and i + 1 < len(argv):
            return argv[i + 1] == "0"
        if a.startswith(("--dist-graph=", "--dp-graph=")):
            return a.split("=", 1)[1] == "0"
    return False


def check_world(args) -> str | None:
    """Errors that must stop the run before any GPU work (None = go)."""
    if args.gpus < 1:
        return f"--gpus must be >= 1 (got {args.gpus})"
    if _in_torchrun():
        world = int(os.environ["WORLD_SIZE"])
        if world != args.gpus:
            return f"torchrun started WORLD_SIZE={world} ranks but --gpus {args.gpus}"
    if not args.shared_gpu and args.gpus > 1:
        have = torch.cuda.device_count()  # counts devices without initialising HIP
        if args.gpus > have:
            return f"--gpus {args.gpus} but this node has {have} GPU(s) (use --shared-gpu for a one-GPU rehearsal)"
    return None


def rank_devices(info, comm=None):
    """Per rank: its device index and name, RCCL's own device / rank / count of the communicator, and
    HIP_VISIBLE_DEVICES -- gathered to rank 0 (collective)."""
    mine = {"rank": info.rank, "device": str(info.device),
            "visible": os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")}
    if info.device.type == "cuda":
        props = torch.cuda.get_device_properties(info.device)
        mine["name"] = props.name
        mine["uuid"] = str(getattr(props, "uuid", ""))[:36] or None
    if comm is not None and hasattr(comm, "device_index"):
        mine.update(rccl_device=comm.device_index(), rccl_rank=comm.user_rank())
    if info.world_size <= 1:
        return [mine]
    import torch.distributed as tdist

    everyone = [None] * info.world_size
    tdist.all_gather_object(everyone, mine)
    return everyone


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    bad = check_world(args)
    if bad:
        print(f"[bench] {bad}", file=sys.stderr)
        return 3
    if args.gpus > 1 and not _in_torchrun():
        return launch_ranks(args.gpus, argv)  # before anything touches the GPU in this process
    from sparse_coding__amd.parallel.dist import init_distributed, shutdown

    info = init_distributed(None if args.dist_backend == "auto" else args.dist_backend,
                            device="cuda:0" if args.shared_gpu else None, force=args.force_dist)
    if not torch.cuda.is_available():
        print("bench.py needs an MI355X (torch.cuda.is_available() is False)", file=sys.stderr)
        return 2
    device = info.device
    torch.manual_seed(0)
    from sparse_coding__amd.models.signatures import FunctionalSAE, FunctionalTiedSAE

    sig = FunctionalSAE if args.kind == "untied" else FunctionalTiedSAE
    n = args.d * args.ratio
    l1s = np.logspace(-4, -2, args.models)
    models = [sig.init(args.d, n, float(l1), device=device) for l1 in l1s]
    ring, held_out = build_ring(args, device)
    B = args.batch

    distributed = info.world_size > 1 or args.force_dist
    if args.dp_chunks is None:
        args.dp_chunks = 2 if info.world_size > 1 else 1
    from sparse_coding__amd.parallel import comm_model

    shape = comm_model.StepShape(models=args.models, n=n, d=args.d, batch=B, t1_ms=T1_MS,
                                 untied=args.kind == "untied", es_ms=dict(ES_MS))
    # N > 1: this node's own collective rates at the step's payloads replace the link model's constants
    # (reported as "comm_calibration")
    calib = compute_calib = None
    if info.world_size > 1 and not args.no_comm_calibration:
        calib = comm_model.calibrate(info, shape)
        try:
            compute_calib = calibrate_compute(info, args, sig, shape)
        except Exception as exc:  # the constants stay; the failure is on record
            compute_calib = {"error": repr(exc)}
    par = args.parallelism
    if par == "auto":
        # N > 1: the mode the per-N comm/compute model predicts fastest (ensemble-axis sharding at
        # the headline config: it moves the batch, not 67 MB of gradients per step)
        par = comm_model.best_mode(info.world_size, shape, args.dp_chunks) if distributed else "dp"
    if not distributed:
        par = "dp"  # one GPU: the plain fused step (no collectives)
    if args.grad_dtype is None:
        args.grad_dtype = "bf16" if par == "zero1" else "fp32"
    grad_dtype = torch.bfloat16 if args.grad_dtype == "bf16" else torch.float32
    if par == "es" and args.models % info.world_size:
        print(f"[bench] --parallelism es needs models % N == 0 ({args.models} models, N={info.world_size})",
              file=sys.stderr)
        return 3

    # N > 1: every multi-rank phase runs under the watchdog (a hang exits HANG_RC; launch_ranks relaunches)
    wd = Watchdog(info, distributed and args.watchdog_scale > 0, args.watchdog_scale or 1.0)
    runner, tiling, warm = ready_runner(par, args, info, sig, models, ring, device, grad_dtype, wd=wd)
    if runner.fallback is None and args.fallback_reason:
        runner.fallback = args.fallback_reason
    wd.arm("timed", WATCHDOG_S["timed"])
    ms, value = warm_and_time(runner, tiling, warm, args, info, B)

    quality = None
    trained = args.warmup + args.steps
    wd.arm("eval", WATCHDOG_S["eval"])
    if not args.no_eval:
        if trained < args.quality_steps:  # untimed: train on toward convergence before evaluating
            from sparse_coding__amd.engine.graph_plan import chunks

            runner.run(chunks(args.quality_steps - trained, tiling.group))
            trained = args.quality_steps
        runner.finish()
        torch.cuda.synchronize()
        lds = runner.dicts()  # collective in the sharded mode: every rank takes part
        if info.is_main:
            quality = fvu_l0(lds, held_out.float())
    runner.finish()
    torch.cuda.synchronize()
    # cross-rank check of the run just timed (collective): replicas identical (dp / zero1) or the same
    # global batches on every rank (es)
    wd.arm("checks", WATCHDOG_S["checks"])
    consistency = runner.consistency() if distributed and runner.consistency is not None else None
    devices = rank_devices(info, runner.comm)
    rccl_ranks = runner.comm.count() if runner.comm is not None and hasattr(runner.comm, "count") else None
    runner.close()

    rec = None
    if info.is_main:
        rec = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "activations/s",
            "n_gpus": info.world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "gpu_event_ms_per_step": (round(runner.gpu_event_ms, 4)
                                      if getattr(runner, "gpu_event_ms", None) is not None else None),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / BASELINE_ACT_PER_S, 2),
            "dtype": "bf16",
            "data": "synthetic (sparse mixture of 4096 unit-norm features, Pythia-70m d_model=512 shape, "
                    f"rows scaled to mean norm {args.act_norm}; random-init SAE weights)",
            "config": {
                "model": f"pythia-70m-resid-sae-ensemble ({args.kind}, d=512, ratio={args.ratio}, "
                         f"{args.models} models, l1=logspace(-4,-2,{args.models}))",
                "global_batch": B * info.world_size,
                "seq_len": None,
                "per_gpu_batch": B,
                "parallelism": f"{par}{info.world_size}",
                "engine": args.engine,
                "dp_chunks": args.dp_chunks if par in ("dp", "zero1") and distributed else None,
                "grad_allreduce_dtype": args.grad_dtype,
            },
            # ring-collective bytes each GPU sends per step in this mode (analytic; 0 on one GPU)
            "comm_bytes_per_gpu_per_step": comm_bytes(par, args, info.world_size) if distributed else 0,
            # parallel/comm_model.py: predicted per-GPU step of every mode at this N (link model +
            # overlap model; the measured ms_per_step above is the check on it)
            "predicted_ms_per_step": {m: comm_model.predict(m, info.world_size, shape, args.dp_chunks)["ms_per_step"]
                                      for m in ("dp", "zero1", "es")} if distributed else None,
            "comm_bytes_other_modes": {m: comm_bytes(m, args, max(info.world_size, 8)) for m in ("dp", "zero1", "es")},
            "comm_calibration": calib,
            "compute_calibration": compute_calib,
            "model_activations_per_s": round(value * args.models, 1),
            "baseline_note": "vs_baseline divides by BASELINE.md row 12 (reference math, same shapes, "
                             "1.86k act/s, 8-vCPU sandbox); no published GPU throughput exists.  "
                             "vs_eager_same_box divides by this repo's PyTorch-eager vmap(grad)+Adam "
                             "engine on the same MI355X (profiles/bench_eager_r2.json)",
            # how the steps were cut into HIP graph replays: all graphs captured + uploaded before
            # warmup; warm_covered = the warmup replayed every timed graph first (engine/graph_plan.py)
            "settle": getattr(runner, "settle", None),
            "graph_replays": {"timed": list(tiling.timed), "warmup": list(tiling.warm),
                              "warm_covered": tiling.covered} if par == "dp" and not distributed
            and not args.no_graph and args.engine == "fused" else None,
            "vs_eager_same_box": round(value / (EAGER_SAME_BOX_ACT_PER_S * info.world_size), 2)
            if EAGER_SAME_BOX_ACT_PER_S and args.engine == "fused" and args.d == 512 and args.ratio == 4
            and args.models == 8 and B == 2048 else None,
        }
        rec["collectives"] = {
            "path": PATH_NAMES.get(runner.path, runner.path) if distributed else PATH_NAMES["single"],
            "fallback": runner.fallback,
            "process_group": {"backend": info.backend, "ranks": info.world_size},
            # the native communicator's own count (ncclCommCount), None when no native comm ran
            "rccl_ranks": rccl_ranks,
            "rank_devices": devices,
            "consistency": consistency,
        }
        if quality is not None:
            rec["fvu_at_l0"] = [{"l1": float(l), "l0": round(a, 2), "fvu": round(b, 4)}
                                for l, (a, b) in zip(l1s, quality)]
            rec["fvu_eval"] = {"train_steps": trained, "held_out_rows": int(held_out.shape[0]),
                               "act_norm": args.act_norm}
        wd.pending = rec  # the headline is measured: a hang from here on still emits it

    # N > 1: also time the other multi-GPU strategy on the same models (untimed for the
    # headline; reported under "alt_parallelism" so both the gradient all-reduce path --
    # BASELINE config 3's mechanism -- and the ensemble-sharded path are on record)
    if distributed and args.compare_parallelism and args.models % info.world_size == 0:
        other = "dp" if par in ("es", "zero1") else "es"
        alt_models = [sig.init(args.d, n, float(l1), device=device) for l1 in l1s]
        alt = {"parallelism": f"{other}{info.world_size}",
               "predicted_ms_per_step": comm_model.predict(other, info.world_size, shape, args.dp_chunks),
               "dp_chunks": args.dp_chunks if other == "dp" else None,
               "comm_bytes_per_gpu_per_step": comm_bytes(other, args, info.world_size)}
        if rec is not None:
            rec["alt_parallelism"] = dict(alt, value=None, ms_per_step=None, error="did not finish (watchdog)")
        try:
            alt_runner, a_tiling, a_warm = ready_runner(other, args, info, sig, alt_models, ring, device, grad_dtype,
                                                        wd=wd, tag="alt-")
            wd.arm("alt-timed", WATCHDOG_S["alt"])
            a_ms, a_value = warm_and_time(alt_runner, a_tiling, a_warm, args, info, B)
            alt_runner.finish()
            torch.cuda.synchronize()
            alt.update(value=round(a_value, 1), ms_per_step=round(a_ms, 4),
                       collective_path=PATH_NAMES.get(alt_runner.path, alt_runner.path),
                       fallback=alt_runner.fallback,
                       consistency=alt_runner.consistency() if alt_runner.consistency is not None else None)
            alt_runner.close()
        except Exception as exc:  # the headline run above stands on its own; the failure is on record
            print(f"[bench] alt parallelism {other} failed: {exc!r}", file=sys.stderr)
            alt.update(value=None, ms_per_step=None, error=repr(exc))
        if rec is not None:
            rec["alt_parallelism"] = alt

    if rec is not None:
        wd.pending = None
        _emit(json.dumps(rec))
    wd.arm("shutdown", WATCHDOG_S["shutdown"])
    shutdown(info)
    wd.disarm()
    return 0


_JSON_FD = None


def _keep_stdout_for_json():
    """The driver reads ONE JSON line from rank 0's stdout, but native libraries print there too (RCCL's
    version banner when a communicator is created): point fd 1 at stderr for everything else and
    keep a private copy of the original stdout for the result line."""
    global _JSON_FD
    if _JSON_FD is None:
        sys.stdout.flush()
        _JSON_FD = os.dup(1)
        os.dup2(2, 1)


def _emit(line: str):
    if _JSON_FD is None:
        print(line, flush=True)
        return
    os.write(_JSON_FD, (line + "\n").encode())


if __name__ == "__main__":
    _keep_stdout_for_json()
    sys.exit(main())
