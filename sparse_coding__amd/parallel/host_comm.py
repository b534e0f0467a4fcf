"""``HostComm``: ``RcclComm``'s interface over a host process group (gloo), staged through host memory.

The graphed data-parallel and ensemble-sharded steps (``parallel/graphed.py``) are written against a
communicator object with ``all_reduce / reduce_scatter / all_gather / all_to_all / broadcast / join``
(``parallel/rccl.py``).  RCCL refuses two ranks on one GPU, so on a one-GPU box (and anywhere the
job runs over gloo) those steps could only ever run at world size 1, where every ``world > 1``
branch is skipped.  ``HostComm`` runs the same collectives through ``torch.distributed`` on CPU
copies of the device buffers: every call synchronises the device, moves the operand to the host,
runs the gloo collective and copies the result back.  It is NOT capturable (``capturable = False``:
the graphed classes then run their step sequence eagerly) and it is slow; it exists so the
multi-rank logic -- shard bounds, in-place gathers, owner sums, event plumbing -- executes and can
be compared against single-process training (``tests/test_graphed_multirank_gpu.py``).

Reference: the DDP experiment's gloo process group (``experiments/huge_batch_size.py:337-345``).
"""

from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from .dist import DistInfo

# gloo's reductions run in fp32 here (bf16 SUM support varies by build); data movement ops ship bytes
_REDUCE_UP = {torch.bfloat16: torch.float32, torch.float16: torch.float32}


class HostComm:
    capturable = False

    def __init__(self, info: DistInfo, group=None):
        if info.world_size > 1 and not dist.is_initialized():
            raise RuntimeError("HostComm needs the default process group")
        self.info, self.group = info, group
        self.world, self.rank = max(1, info.world_size), info.rank
        self.device = torch.device(info.device)
        self.stream = torch.cuda.current_stream(self.device) if self.device.type == "cuda" else None
        self.calls = {}  # collective name -> count (tests / reports: which collectives ran)

    def _note(self, name: str):
        self.calls[name] = self.calls.get(name, 0) + 1

    @staticmethod
    def _host(t: torch.Tensor, dtype=None) -> torch.Tensor:
        """A host copy (synchronises the producer's stream through the device-to-host copy)."""
        h = t.detach().to("cpu", copy=True)
        return h.to(dtype) if dtype is not None and h.dtype != dtype else h

    @staticmethod
    def _bytes(t: torch.Tensor) -> torch.Tensor:
        return t.contiguous().reshape(-1).view(torch.uint8)

    # ------------------------------------------------------------------ collectives (RcclComm API)
    def all_reduce(self, t: torch.Tensor, overlap: bool = False, fork: bool = True):
        """In-place SUM over ranks."""
        self._note("all_reduce")
        if self.world == 1:
            return None
        h = self._host(t, _REDUCE_UP.get(t.dtype))
        dist.all_reduce(h, group=self.group)
        t.copy_(h.to(t.dtype))
        return None

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, overlap: bool = False, fork: bool = True):
        """out = this rank's 1/N block of the SUM of ``inp`` over ranks."""
        if inp.numel() != self.world * out.numel() or inp.dtype != out.dtype:
            raise ValueError("reduce_scatter: inp must hold world x out elements of the same dtype")
        self._note("reduce_scatter")
        h = self._host(inp.reshape(-1), _REDUCE_UP.get(inp.dtype))
        if self.world > 1:
            dist.all_reduce(h, group=self.group)
        k = out.numel()
        out.view(-1).copy_(h[self.rank * k:(self.rank + 1) * k].to(out.dtype))
        return None

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, overlap: bool = False, fork: bool = True):
        """out = concat over ranks of ``inp`` (rank-major); ``inp`` may be out's own block (in place)."""
        if out.numel() != self.world * inp.numel() or inp.dtype != out.dtype:
            raise ValueError("all_gather: out must hold world x inp elements of the same dtype")
        self._note("all_gather")
        h = self._bytes(self._host(inp))
        parts = [torch.empty_like(h) for _ in range(self.world)]
        if self.world > 1:
            dist.all_gather(parts, h, group=self.group)
        else:
            parts = [h]
        out.view(-1).view(torch.uint8).copy_(torch.cat(parts))
        return None

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, overlap: bool = False, fork: bool = True):
        """out[j] = rank j's inp block for this rank (N equal blocks)."""
        if out.numel() != inp.numel() or inp.numel() % self.world or inp.dtype != out.dtype:
            raise ValueError("all_to_all: equal-size buffers of N blocks")
        self._note("all_to_all")
        h = self._bytes(self._host(inp))
        r = torch.empty_like(h)
        if self.world > 1:
            dist.all_to_all_single(r, h, group=self.group)
        else:
            r.copy_(h)
        out.view(-1).view(torch.uint8).copy_(r)
        return None

    def broadcast(self, t: torch.Tensor, root: int = 0, overlap: bool = False, fork: bool = True):
        self._note("broadcast")
        if self.world == 1:
            return None
        h = self._bytes(self._host(t))
        dist.broadcast(h, src=int(root), group=self.group)
        t.view(-1).view(torch.uint8).copy_(h)
        return None

    def count(self) -> int:
        return self.world

    def join(self, stream: Optional[torch.cuda.Stream] = None):
        """Nothing in flight: every call above completed before it returned."""

    def close(self):
        pass
