"""HBM-resident activation ring buffer.

The reference keeps each 2 GiB activation chunk in host memory and, per
batch, gathers random rows on the CPU and copies them to the GPU
(``big_sweep.py:170``, ``cluster_runs.py:101-102``).  On MI355X the activations
live in HBM (288 GB per GPU holds ~280 M rows of d=512 bf16): producers (the
synthetic generator, the harvester, the chunk loader) append rows, and the
trainer draws batches with an on-device random gather -- no host round trip
per step.  Sampling is without replacement within an epoch (a device-side
permutation), matching ``BatchSampler(RandomSampler(...))`` in the reference.
"""

from __future__ import annotations

import math
from typing import Callable, Iterable, Optional

import torch


def rows_for_budget(d: int, bytes_budget: int, dtype=torch.bfloat16) -> int:
    return int(bytes_budget // (d * torch.empty((), dtype=dtype).element_size()))


def hbm_budget(fraction: float = 0.8, device=None) -> int:
    """Bytes of free device memory times ``fraction`` (sizes the ring for 288 GB parts)."""
    free, _ = torch.cuda.mem_get_info(device)
    return int(free * fraction)


class DeviceRing:
    def __init__(self, capacity: int, d: int, device="cuda", dtype=torch.bfloat16, seed: int = 0):
        self.capacity = int(capacity)
        self.d = d
        self.device = torch.device(device)
        self.dtype = dtype
        self.buf = torch.empty(self.capacity, d, device=self.device, dtype=dtype)
        self.size = 0      # valid rows
        self.head = 0      # next write position
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed)
        self._perm: Optional[torch.Tensor] = None
        self._cursor = 0
        self.epoch = 0

    @classmethod
    def from_hbm(cls, d: int, fraction: float = 0.5, max_rows: Optional[int] = None, device="cuda", **kw):
        rows = rows_for_budget(d, hbm_budget(fraction, device))
        if max_rows:
            rows = min(rows, max_rows)
        return cls(rows, d, device=device, **kw)

    # ------------------------------------------------------------------ producers
    def push(self, rows: torch.Tensor):
        """Append rows (any dtype/device); wraps around, overwriting the oldest rows."""
        rows = rows.reshape(-1, self.d)
        n = rows.shape[0]
        if n > self.capacity:
            rows = rows[-self.capacity:]
            n = self.capacity
        first = min(n, self.capacity - self.head)
        self.buf[self.head:self.head + first].copy_(rows[:first], non_blocking=True)
        if n > first:
            self.buf[: n - first].copy_(rows[first:], non_blocking=True)
        self.head = (self.head + n) % self.capacity
        self.size = min(self.capacity, self.size + n)
        self._perm = None

    def fill(self, producer: Callable[[], torch.Tensor], rows: Optional[int] = None):
        """Call ``producer()`` until ``rows`` (default: capacity) rows have been pushed."""
        target = self.capacity if rows is None else min(rows, self.capacity)
        pushed = 0
        while pushed < target:
            chunk = producer()
            chunk = chunk[: target - pushed]
            self.push(chunk)
            pushed += chunk.shape[0]
        return self

    # ------------------------------------------------------------------ consumer
    def _new_epoch(self):
        self._perm = torch.randperm(self.size, device=self.device, generator=self.gen)
        self._cursor = 0
        self.epoch += 1

    def ensure_permutation(self):
        """Draw the current epoch's permutation now if none exists (setup time, not first use)."""
        if self._perm is None and self.size:
            self._new_epoch()
        return self

    def sample(self, batch_size: int, out: Optional[torch.Tensor] = None, return_index: bool = False):
        """Random batch (without replacement within an epoch), gathered on device.
        With ``return_index`` also returns the ring row indices ``[batch_size]``."""
        return self.sample_shard(batch_size, 0, 1, out=out, return_index=return_index)

    def sample_shard(self, batch_size: int, rank: int, world: int, out=None, return_index: bool = False):
        """Data-parallel sampling: every rank draws the same global permutation slice and
        keeps its own contiguous shard (DistributedSampler semantics on device)."""
        if self.size == 0:
            raise RuntimeError("ring is empty")
        if self._perm is None or self._cursor + batch_size * world > self._perm.numel():
            self._new_epoch()
        idx = self._perm[self._cursor + rank * batch_size:self._cursor + (rank + 1) * batch_size]
        self._cursor += batch_size * world
        if (self.buf.is_cuda and (self.buf[0].numel() * self.buf.element_size()) % 16 == 0
                and idx.dtype == torch.int64 and _kernels_available()):
            from ..ops.rows import gather_rows  # one wave per row (HIP); torch index_select elsewhere

            # (indices come from this ring's own permutation of [0, size): always in bounds)
            rows = gather_rows(self.buf, idx, out=out)
        else:
            rows = self.buf.index_select(0, idx) if out is None else torch.index_select(self.buf, 0, idx, out=out)
        return (rows, idx) if return_index else rows

    def sample_shard_steps(self, batch_size: int, rank: int, world: int, steps: int, out: torch.Tensor):
        """This rank's rows of the next ``steps`` data-parallel steps into ``out`` [steps * batch_size, d]
        in one gather: step s's shard is the same permutation block ``sample_shard`` would return at
        its s-th call.  When the group would run past the epoch's permutation, a new epoch starts at
        the group (up to ``steps - 1`` global batches of the old one are skipped -- every epoch is
        still a without-replacement pass)."""
        if self.size == 0:
            raise RuntimeError("ring is empty")
        steps = int(steps)
        need = batch_size * world * steps
        if out.shape[0] != steps * batch_size:
            raise ValueError(f"out has {out.shape[0]} rows, need {steps * batch_size}")
        if self._perm is None or self._cursor + need > self._perm.numel():
            self._new_epoch()
            if need > self._perm.numel():
                raise ValueError(f"{steps} steps of {batch_size} x {world} rows exceed the ring ({self.size} rows)")
        base = self._cursor + rank * batch_size
        if (self.buf.is_cuda and (self.buf[0].numel() * self.buf.element_size()) % 16 == 0
                and _kernels_available()):
            from ..ops.rows import gather_rows_blocks

            gather_rows_blocks(self.buf, self._perm, base, batch_size * world, batch_size, out)
        else:
            idx = self._perm[self._cursor:self._cursor + need].view(steps, world, batch_size)[:, rank].reshape(-1)
            torch.index_select(self.buf, 0, idx, out=out)
        self._cursor += need
        return out

    def graph_source(self, batch_size: int, rank: int = 0, world: int = 1) -> "RingGraphSource":
        """A batch source whose fetch can run INSIDE a training engine's HIP graph (see
        ``RingGraphSource``); it walks this ring's permutations like ``sample`` (``sample_shard``
        for a data-parallel rank)."""
        return RingGraphSource(self, batch_size, rank, world)

    def batches_per_epoch(self, batch_size: int) -> int:
        return self.size // batch_size

    def view(self) -> torch.Tensor:
        return self.buf[: self.size]


class RingGraphSource:
    """In-graph batch fetch from a ``DeviceRing`` (single process).

    Step t of an engine reads rows ``perm[(t - ep0) * B : (t - ep0 + 1) * B]`` of a permutation kept
    in a persistent device buffer; t is the engine's device step counter (advanced inside the
    captured step), ep0 a device scalar.  Between replays ``prepare(t)`` rolls a fresh permutation
    into the same buffer (and sets ep0 = t) when the epoch is exhausted -- the same
    without-replacement epochs as ``DeviceRing.sample``.  The fetch itself is one gather kernel
    that is part of the step's graph, so no plain launch sits between graph replays.

    Data parallel (``rank`` of ``world``): every rank walks the same permutation (same ring seed) and
    step t of rank r reads the block ``perm[((t - ep0) N + r) B, +B)`` -- its shard of the global batch
    of N B rows, the ``DeviceRing.sample_shard`` (DistributedSampler) semantics."""

    def __init__(self, ring: DeviceRing, batch_size: int, rank: int = 0, world: int = 1):
        if ring.size < batch_size * world:
            raise ValueError("ring holds fewer rows than one global batch")
        self.ring, self.B = ring, int(batch_size)
        self.rank, self.world = int(rank), int(world)
        dev = ring.device
        # the permutation covers the rows valid at attach time (the captured gather reads this
        # buffer, so its size is fixed); rows appended later are walked after ``resize()``
        self.rows = int(ring.size)
        self.perm = torch.empty(self.rows, device=dev, dtype=torch.int64)
        self.ep0 = torch.zeros(1, device=dev, dtype=torch.int32)
        self._ep0_host = None  # step at which the current permutation started

    def prepare(self, step: int, steps: int = 1):
        """Host bookkeeping before replaying steps ``step .. step + steps - 1``: a new permutation
        when they would run past the current one (a multi-step replay may start the next epoch
        up to ``steps - 1`` batches early: every epoch is still a without-replacement pass)."""
        if self._ep0_host is None or (step - self._ep0_host + steps) * self.B * self.world > self.perm.numel():
            self.perm.copy_(torch.randperm(self.rows, device=self.ring.device, generator=self.ring.gen))
            self.ep0.fill_(int(step))
            self._ep0_host = int(step)
            self.ring.epoch += 1
        # every in-graph fetch of these steps -- the gather kernels and the fused tail's next-batch
        # fetch (row (t + 1 - ep0) B N + r for t < step + steps - 1) -- indexes inside the permutation
        # (the kernels clamp out-of-range indices to row 0 silently; this is the host-side check)
        if (step - self._ep0_host + steps) * self.B * self.world > self.perm.numel() or step < self._ep0_host:
            raise RuntimeError(f"steps {step}..{step + steps - 1} do not fit the ring permutation "
                               f"({self.perm.numel()} rows from step {self._ep0_host}, {self.B * self.world} per step)")

    def tail_gather(self, out: torch.Tensor):
        """(ring buffer, permutation, epoch start, out): what a fused step tail needs to fetch the NEXT
        step's rows into ``out`` (csrc/adam.hip step_tail_kernel, row ``(t + 1 - ep0) * B + r``);
        None for a data-parallel shard (the tail's fetch has no rank offset)."""
        if self.world != 1:
            return None
        return (self.ring.buf, self.perm, self.ep0, out)

    def gather(self, out: torch.Tensor, step_dev: torch.Tensor):
        """The capturable fetch: ``out`` [B, ...] <- this step's rows."""
        from ..ops.rows import gather_rows_perm

        return gather_rows_perm(self.ring.buf, self.perm, step_dev, self.ep0, out, stride=self.B * self.world,
                                offset=self.rank * self.B)

    def gather_steps(self, out: torch.Tensor, step_dev: torch.Tensor):
        """The capturable fetch of a multi-step group: ``out`` [s, B, ...] <- this rank's rows of steps
        t .. t+s-1 (one launch)."""
        from ..ops.rows import gather_rows_perm

        s = out.shape[0]
        if out.shape[1] != self.B or not out.is_contiguous():
            raise ValueError(f"out must be contiguous [s, {self.B}, ...]")
        return gather_rows_perm(self.ring.buf, self.perm, step_dev, self.ep0, out.view(s * self.B, *out.shape[2:]),
                                stride=self.B * self.world, offset=self.rank * self.B, inner=self.B, ostride=self.B)

    def gather_into_global(self, glob: torch.Tensor, step_dev: torch.Tensor):
        """The capturable fetch of a multi-step group for an in-place all-gather: ``glob`` [s, N B, ...]
        (one global batch per step); this rank's rows of steps t .. t+s-1 go straight into its slots
        ``glob[k, rank B : (rank + 1) B]`` in ONE launch (no send buffer, no copy)."""
        from ..ops.rows import gather_rows_perm

        s, NB = glob.shape[0], glob.shape[1]
        if NB != self.B * self.world or not glob.is_contiguous():
            raise ValueError(f"glob must be contiguous [s, {self.B * self.world}, ...]")
        flat = glob.view(s * NB, *glob.shape[2:])
        lo = self.rank * self.B
        out = flat[lo: (s - 1) * NB + lo + self.B]
        return gather_rows_perm(self.ring.buf, self.perm, step_dev, self.ep0, out, stride=NB, offset=lo,
                                inner=self.B, ostride=NB)


def _kernels_available() -> bool:
    from ..ops import _lib

    return _lib.available()
