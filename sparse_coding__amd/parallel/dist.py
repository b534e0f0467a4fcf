"""Process-group bootstrap: one process per GPU, RCCL ("nccl" backend on ROCm) over xGMI.

Reads the torchrun environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
MASTER_PORT).  Without it the job is a single process.  CPU-only runs (tests,
this container) use gloo, so the distributed logic is exercised without a GPU.
"""

from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def enabled(self) -> bool:
        return self.world_size > 1


def init_distributed(backend: str | None = None, timeout_s: int = 600, device=None, force: bool = False) -> DistInfo:
    """``device`` overrides the per-rank device (e.g. several gloo ranks sharing one GPU in a test).
    ``force`` creates the process group even for a single process (rehearses the collective
    code paths with real RCCL on a one-GPU box)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_cuda = torch.cuda.is_available() and backend != "gloo"
    if device is not None:
        device = torch.device(device)
        if device.type == "cuda":
            torch.cuda.set_device(device)
    elif use_cuda:
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    if (world > 1 or force) and not dist.is_initialized():
        os.environ.setdefault("MASTER_PORT", "29511")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # fail fast: a dead or hung rank aborts the collective (and the job) after
        # `timeout_s` instead of hanging every other rank
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        be = backend or ("nccl" if use_cuda else "gloo")
        kw = dict(backend=be, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if be == "nccl":
            kw["device_id"] = device
            if os.environ.get("SC_RCCL_HIGH_PRIORITY", "1") not in ("", "0"):
                # RCCL's internal stream at high priority: the collectives that run under the
                # step's GEMMs (ensemble-sharded batch all-gather, chunked DP all-reduce) get
                # their workgroups dispatched ahead of the compute stream's
                opts = dist.ProcessGroupNCCL.Options()
                opts.is_high_priority_stream = True
                kw["pg_options"] = opts
        dist.init_process_group(**kw)
        return DistInfo(rank, world, local, device, be)
    if dist.is_initialized():
        return DistInfo(dist.get_rank(), dist.get_world_size(), local, device, dist.get_backend())
    return DistInfo(0, 1, 0, device, "none")


def barrier(info: DistInfo):
    if info.enabled:
        if info.backend == "nccl":
            dist.barrier(device_ids=[info.local_rank])
        else:
            dist.barrier()


def all_reduce_max(value: float, info: DistInfo) -> float:
    if not info.enabled:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=info.device if info.backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def broadcast_(t: torch.Tensor, info: DistInfo, src: int = 0):
    if info.enabled:
        dist.broadcast(t, src=src)
    return t


def shutdown(info: DistInfo):
    if dist.is_initialized():
        dist.destroy_process_group()
