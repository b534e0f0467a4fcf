"""``DelayedSimComm``: a capturable stand-in for ``RcclComm`` that makes missing stream joins visible.

At one RCCL rank every collective is a near no-op that completes almost instantly on the
communicator's stream, so a consumer that forgot to wait for a collective's event (``red_ev``,
``gath_ev``, an ES batch gather) still reads the right bytes and every one-rank test passes; the
gloo rehearsal comm (``host_comm.HostComm``) is synchronous, so it cannot expose a missing join
either.  This communicator runs on ONE GPU inside ``torch.cuda.graph`` capture exactly like the
native one -- its own stream, events returned for ``overlap=True``, ``join()`` -- but

* every collective sits behind a spin kernel of ``delay_us`` on the comm stream, so the result lands
  long after the producer's next kernels, and
* it simulates ``world`` IDENTICAL replicas of the calling rank (rank ``rank``): ``all_reduce``
  multiplies by ``world`` (the SUM of ``world`` equal tensors; with the data-parallel
  ``grad_scale = 1/world`` the update equals one rank's), ``reduce_scatter`` returns ``world`` times
  this rank's block, ``all_gather`` / ``all_to_all`` fill every rank's block with this rank's
  (identical replicas hold identical blocks), ``broadcast`` keeps the data.

A consumer that does not wait on the right event reads the pre-collective bytes (or races the
in-place update) and its result differs from the same sequence run with ``delay_us=0`` and
``sync=True`` (every collective on the current stream, fully ordered): that comparison is the test
(``tests/test_sim_comm_gpu.py``).  Not meant for training; the reduce-scatter / all-gather of
ZeRO-1 row shards is NOT a faithful simulation (other ranks own other rows), so ZeRO-1 stays covered
by the multi-rank gloo tests.  Reference: ``experiments/huge_batch_size.py:337-363`` (the DDP ranks
the real communicator serves).
"""

from __future__ import annotations

from typing import Optional

import torch


class DelayedSimComm:
    capturable = True

    def __init__(self, device, world: int = 2, rank: int = 0, delay_us: float = 50.0, sync: bool = False,
                 clock_ghz: float = 2.4):
        if world < 1 or not 0 <= rank < world:
            raise ValueError(f"need 0 <= rank < world (got rank {rank}, world {world})")
        self.device = torch.device(device)
        self.world, self.rank = int(world), int(rank)
        self.sync = bool(sync)
        # torch.cuda._sleep spins for a number of shader-clock cycles (capturable: a plain kernel)
        self.cycles = int(max(0.0, delay_us) * 1e3 * clock_ghz)
        self.stream = (torch.cuda.current_stream(self.device) if self.sync
                       else torch.cuda.Stream(self.device))
        self.calls = {}

    # ------------------------------------------------------------------ stream plumbing (RcclComm's)
    def join(self, stream: Optional[torch.cuda.Stream] = None):
        if not self.sync:
            (stream or torch.cuda.current_stream(self.device)).wait_stream(self.stream)

    def _run(self, name: str, fn, overlap: bool, fork: bool = True):
        self.calls[name] = self.calls.get(name, 0) + 1
        if self.sync:  # the reference ordering: on the producer's stream, nothing in flight
            fn()
            return None
        cur = torch.cuda.current_stream(self.device)
        if fork:  # (RcclComm._run: the 2nd.. collectives of a back-to-back batch do not fork again)
            self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            if self.cycles:
                torch.cuda._sleep(self.cycles)
            fn()
        if not overlap:
            cur.wait_stream(self.stream)
            return None
        ev = torch.cuda.Event()
        ev.record(self.stream)
        return ev

    # ------------------------------------------------------------------ collectives (N identical replicas)
    def all_reduce(self, t: torch.Tensor, overlap: bool = False, fork: bool = True):
        return self._run("all_reduce", lambda: t.mul_(self.world) if self.world > 1 else None, overlap, fork)

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, overlap: bool = False, fork: bool = True):
        if inp.numel() != self.world * out.numel() or inp.dtype != out.dtype:
            raise ValueError("reduce_scatter: inp must hold world x out elements of the same dtype")
        k = out.numel()

        def fn():
            torch.mul(inp.reshape(-1)[self.rank * k:(self.rank + 1) * k], self.world, out=out.view(-1))

        return self._run("reduce_scatter", fn, overlap, fork)

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, overlap: bool = False, fork: bool = True):
        if out.numel() != self.world * inp.numel() or inp.dtype != out.dtype:
            raise ValueError("all_gather: out must hold world x inp elements of the same dtype")
        k = inp.numel()

        def fn():
            src = inp.reshape(-1)
            flat = out.view(-1)
            for j in range(self.world):
                dst = flat[j * k:(j + 1) * k]
                if dst.data_ptr() != src.data_ptr():  # (in place: this rank's block is already there)
                    dst.copy_(src)

        return self._run("all_gather", fn, overlap, fork)

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, overlap: bool = False, fork: bool = True):
        if out.numel() != inp.numel() or inp.numel() % self.world or inp.dtype != out.dtype:
            raise ValueError("all_to_all: equal-size buffers of N blocks")
        k = inp.numel() // self.world

        def fn():
            blk = inp.reshape(-1)[self.rank * k:(self.rank + 1) * k]
            out.view(self.world, k).copy_(blk.unsqueeze(0).expand(self.world, k))

        return self._run("all_to_all", fn, overlap, fork)

    def broadcast(self, t: torch.Tensor, root: int = 0, overlap: bool = False, fork: bool = True):
        return self._run("broadcast", lambda: None, overlap, fork)

    def count(self) -> int:
        return self.world

    def close(self):
        torch.cuda.synchronize(self.device)
