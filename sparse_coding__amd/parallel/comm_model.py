"""Per-N communication budget of the multi-GPU SAE ensemble step on one MI355X node (xGMI).

BASELINE config 3 trains an SAE ensemble data-parallel over 8 GPUs with an RCCL gradient all-reduce
(reference DDP experiment: ``experiments/huge_batch_size.py:274, 313, 329``).  For an SAE ensemble
the gradient is as large as the parameters, so whether a data-parallel step can hide its collectives
is a bandwidth question this module answers with explicit numbers, per strategy and GPU count:

* ``dp``    all-reduce of the weight + bias gradients: 2 (N-1)/N x g bytes per GPU;
* ``zero1`` reduce-scatter of the gradients (bf16 transport, fp32 owner accumulation by default) +
            all-gather of the updated bf16 shadows: (N-1)/N x (g + s) bytes, and Adam on 1/N of the rows;
* ``es``    ensemble-axis sharding: all-gather of the batch, (N-1)/N x b bytes; each GPU trains G/N
            models on the N B global batch (same FLOPs, 1/N of the Adam traffic).

Link model.  The 8 MI355X of a node are fully connected by xGMI: every pair has its own link
(7 per GPU), ~64 GB/s per direction measured for one pair by the RCCL rings (the task's 7 x ~153
GB/s is the bidirectional raw rate).  A ring collective over N GPUs built from RCCL's channels can
drive at most N-1 links per GPU at once; ``LINK_EFF`` discounts protocol and scheduling overheads
(RCCL bus bandwidth on xGMI meshes sits well under the raw link sum).  Every number here is an
input of the model, not a measurement of this node -- unless ``calibrate()`` measured the node's own
collectives first (the bench does at N > 1 and reports them): its bus rates then replace the link
model per mode.  The bench prints the prediction next to the measured step so the two can be compared
on the driver's 8-GPU runs.

Overlap model.  ``dp`` with K model chunks overlaps chunk k's all-reduce with chunk k+1's compute
(and, cross-step, the last chunk's with the next step's first chunk): up to (K-1)/K of the step's
compute can hide communication; what exceeds it is exposed.  ``zero1`` overlaps the same way;
``es`` overlaps the next group's batch gather with the current group's replay (fully hidden unless
the gather outlasts the group).
"""

from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Dict, Optional

LINK_GBPS = 64.0     # one xGMI link, one direction, GB/s (RCCL ring measurement, 2 GPUs)
LINKS_PER_GPU = 7    # fully connected 8-GPU node
LINK_EFF = 0.7       # fraction of the summed link rate a ring collective sustains


def bus_gbps(world: int) -> float:
    """Sustained per-GPU collective bandwidth (GB/s) for a ring over ``world`` GPUs."""
    if world <= 1:
        return float("inf")
    return min(world - 1, LINKS_PER_GPU) * LINK_GBPS * LINK_EFF


@dataclass
class StepShape:
    """The ensemble step being distributed: G models of n x d (untied: encoder + decoder), B rows
    per GPU per step, ``t1_ms`` the measured single-GPU step (all G models, B rows)."""
    models: int
    n: int
    d: int
    batch: int
    t1_ms: float
    untied: bool = True
    adam_ms: float = 0.08          # Adam share of t1 (HBM-bound; divides by N under zero1 / es)
    es_ms: Dict[int, float] = field(default_factory=dict)  # measured per-rank ES steps, if any
    bus: Dict[str, float] = field(default_factory=dict)    # measured bus GB/s per mode (calibrate())
    compute_source: str = "constants"  # "measured on this node" once use_measured_compute() ran

    def use_measured_compute(self, world: int, t1_ms: Optional[float], es_ms: Optional[float]):
        """Replace the compute inputs with steps timed on this node (bench.py ``calibrate_compute``):
        ``t1_ms`` = one GPU's step of all G models on B rows (dp / zero1 per-rank layout), ``es_ms`` =
        the ensemble-sharded per-rank layout (G/N models on N B rows).  ``best_mode`` then ranks the
        modes on these numbers instead of the builder box's constants."""
        if t1_ms:
            self.t1_ms = float(t1_ms)
        if es_ms:
            self.es_ms = dict(self.es_ms)
            self.es_ms[world] = float(es_ms)
        if t1_ms or es_ms:
            self.compute_source = "measured on this node"

    @property
    def params(self) -> int:
        return self.models * ((2 if self.untied else 1) * self.n * self.d + self.n)

    @property
    def shadow_bytes(self) -> int:
        return self.models * (2 if self.untied else 1) * self.n * self.d * 2


def bytes_per_gpu(mode: str, world: int, shape: StepShape, grad_bytes_per_elem: int = 4) -> int:
    """Bytes each GPU sends per step (ring collectives)."""
    f = (world - 1) / world if world > 1 else 0.0
    g = shape.params * grad_bytes_per_elem
    if mode == "dp":
        return int(2 * f * g)
    if mode == "zero1":
        return int(f * (g + shape.shadow_bytes))
    if mode == "es":
        return int(f * world * shape.batch * shape.d * 2)  # all-gather of the N B-row global batch
    raise ValueError(mode)


def predict(mode: str, world: int, shape: StepShape, dp_chunks: int = 2,
            grad_bytes_per_elem: Optional[int] = None) -> Dict[str, float]:
    """Predicted per-GPU step (ms) = compute + exposed communication, with its parts."""
    if grad_bytes_per_elem is None:
        grad_bytes_per_elem = 2 if mode == "zero1" else 4  # zero1: bf16 transport by default
    nbytes = bytes_per_gpu(mode, world, shape, grad_bytes_per_elem)
    bw = shape.bus.get(mode) or bus_gbps(world)
    comm_ms = nbytes / (bw * 1e9) * 1e3 if world > 1 else 0.0
    if mode == "es":
        compute = shape.es_ms.get(world, shape.t1_ms - shape.adam_ms * (1 - 1 / world))
        hide = compute  # the next group's gather runs under this group's replay
    elif mode == "zero1":
        compute = shape.t1_ms - shape.adam_ms * (1 - 1 / world)
        hide = compute * (dp_chunks - 1) / dp_chunks if dp_chunks > 1 else 0.0
    else:
        compute = shape.t1_ms
        hide = compute * (dp_chunks - 1) / dp_chunks if dp_chunks > 1 else 0.0
    exposed = max(0.0, comm_ms - hide)
    return {"ms_per_step": round(compute + exposed, 4), "compute_ms": round(compute, 4),
            "comm_ms": round(comm_ms, 4), "exposed_comm_ms": round(exposed, 4),
            "bytes_per_gpu": nbytes, "bus_GBps": round(bw, 1) if world > 1 else None,
            "bus_source": ("measured" if shape.bus.get(mode) else "link model") if world > 1 else None,
            "compute_source": shape.compute_source}


def calibrate(info, shape: StepShape, reps: int = 5) -> Optional[Dict[str, Dict[str, float]]]:
    """Time this node's own collectives at the step's payloads (collective: every rank calls it; N > 1).

    * ``all_gather`` of each rank's B x d bf16 batch (the ``es`` payload);
    * ``all_reduce`` of the fp32 weight + bias gradients (the ``dp`` payload; ``zero1`` moves the same
      ring volume as reduce-scatter + all-gather, so it takes this rate).
    Median of ``reps`` timed runs after two warmups, barrier + device synchronize around each.  Bus
    bandwidth as RCCL reports it: all-reduce 2 (N-1)/N x bytes / t, all-gather (N-1)/N x N x bytes / t.
    Fills ``shape.bus`` (GB/s per mode) and returns the measurements (None on one rank)."""
    import torch
    import torch.distributed as dist

    from .dist import barrier

    if not getattr(info, "enabled", False) or info.world_size <= 1:
        return None
    world = info.world_size
    dev = info.device if info.backend == "nccl" else torch.device("cpu")
    cuda = dev.type == "cuda"

    def timed(fn):
        for _ in range(2):
            fn()
        ts = []
        for _ in range(reps):
            barrier(info)
            if cuda:
                torch.cuda.synchronize(dev)
            t = time.perf_counter()
            fn()
            if cuda:
                torch.cuda.synchronize(dev)
            ts.append(time.perf_counter() - t)
        ts.sort()
        return ts[len(ts) // 2]

    f = (world - 1) / world
    out = {"backend": info.backend}
    x = torch.ones(shape.batch, shape.d, dtype=torch.bfloat16, device=dev)
    parts = [torch.empty_like(x) for _ in range(world)]
    t = timed(lambda: dist.all_gather(parts, x))
    nb = x.numel() * x.element_size()
    out["all_gather"] = {"bytes_per_rank": nb, "ms": round(t * 1e3, 4), "bus_GBps": round(f * world * nb / t / 1e9, 2)}
    g = torch.ones(shape.params, dtype=torch.float32, device=dev)
    t = timed(lambda: dist.all_reduce(g))
    nb = g.numel() * 4
    out["all_reduce"] = {"bytes": nb, "ms": round(t * 1e3, 4), "bus_GBps": round(2 * f * nb / t / 1e9, 2)}
    del x, parts, g
    shape.bus.update({"es": out["all_gather"]["bus_GBps"], "dp": out["all_reduce"]["bus_GBps"],
                      "zero1": out["all_reduce"]["bus_GBps"]})
    return out


def best_mode(world: int, shape: StepShape, dp_chunks: int = 2, allow_es: bool = True) -> str:
    modes = ["dp", "zero1"] + (["es"] if allow_es and shape.models % world == 0 else [])
    return min(modes, key=lambda m: predict(m, world, shape, dp_chunks)["ms_per_step"])


def table(shape: StepShape, worlds=(1, 2, 4, 8), dp_chunks: int = 2) -> Dict[int, Dict[str, Dict[str, float]]]:
    return {w: {m: predict(m, w, shape, dp_chunks) for m in ("dp", "zero1", "es")} for w in worlds}


def main():  # python -m sparse_coding__amd.parallel.comm_model
    import json

    # the headline config: 8 untied SAEs, d = 512, n = 2048, B = 2048 rows per GPU; t1 and the ES
    # per-rank steps from profiles/bench_r3_v5_final.json and profiles/es_projection_r3.jsonl
    shape = StepShape(models=8, n=2048, d=512, batch=2048, t1_ms=0.3064,
                      es_ms={2: 0.285, 4: 0.2714, 8: 0.2621})
    for w, row in table(shape).items():
        print(json.dumps({"N": w, "best": best_mode(w, shape), **row}))


if __name__ == "__main__":
    main()
