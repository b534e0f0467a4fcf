"""Data-parallel (DP / ZeRO-1) fused training with the collectives INSIDE multi-step HIP graphs.

The host-issued data-parallel paths (``parallel/data_parallel.py``, ``parallel/zero.py``) replay a
"grads" and an "update" graph per model chunk and issue the collectives between them through
ProcessGroupNCCL -- four graph replays and their idle gaps per step at two chunks, plus an eager
batch gather.  Here a group of S optimizer steps is ONE graph: per step the rank's batch shard is
fetched from the HBM ring inside the graph (``RingGraphSource`` rank shard, device step counter),
every chunk computes its gradients, its reduction runs on the communicator's own stream
(``parallel/rccl.py``: RCCL enqueued on our stream, captured as graph nodes) while the next chunk
computes, and the chunk's update joins on exactly that reduction's event::

    step s:  fetch x_s | chunk 0 fwd+bwd -> reduce(0) ....................... (comm stream)
                       | update(K-1 of step s-1)     <- waits reduce(K-1, s-1)   (cross-step)
                       | chunk 1 fwd+bwd -> reduce(1) ...
                       | update(0)                   <- waits reduce(0)
    end of group: update(K-1)

``mode="dp"``: all-reduce of each chunk's flat fp32 gradient (pre-scaled by 1/N in the GEMM
epilogues, so the SUM is the global-batch mean).  ``mode="zero1"``: each chunk's dictionary rows
are sharded over ranks -- reduce-scatter of the weight gradients (fp32; or bf16 transport by
all-to-all with fp32 accumulation on the owner), all-reduce of the small bias / extras tail, Adam on
the owned rows only, all-gather of the updated bf16 shadows and row norms (waited on by the chunk's
next compute).  Per model the update is exactly data-parallel Adam on the global batch of N B rows
(reference DDP semantics, ``experiments/huge_batch_size.py:259-345``).
"""

from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import torch

from ..ops import adam as adam_ops

from .dist import DistInfo
from .zero import shard_range


class _Chunk:
    def __init__(self, engine, mode: str, info: DistInfo, grad_dtype):
        e = self.engine = engine
        kind = getattr(e, "kind", None)
        if kind not in ("untied", "tied") or e.learned_center:
            raise NotImplementedError(f"graphed data parallel of engine kind {kind} (learned centre)")
        # Masked ensembles (per-model live sizes, reference sae_ensemble.py:306-442): the compacted
        # launches never write a dead row of the flat gradient (the engine zero-initialises it), so the
        # reductions carry zeros there on every rank, and every update skips dead rows (``live``).
        # the reductions read the flat fp32 gradient buffer: drop any split-K slabs / bf16 copy the
        # engine picked for its own shape (FusedSAEEnsemble(wgrad_split='auto'))
        e.use_flat_grads()
        self.mode = mode
        G, n, d = e.n_models, e.n, e.d
        N = max(1, info.world_size)
        self.world = N
        if mode == "zero1":
            self.lo, self.hi = shard_range(G * n, info.rank, N)
            rows = self.hi - self.lo
            dev = e.device
            self.srcs = [e.g_dec] + ([e.g_enc] if kind == "untied" else [])
            self.shards = [torch.empty(rows, d, device=dev) for _ in self.srcs]
            self.lowp = grad_dtype != torch.float32 and N > 1
            if self.lowp:
                self.send = [torch.empty(G * n * d, device=dev, dtype=grad_dtype) for _ in self.srcs]
                self.recv = [torch.empty(N * rows * d, device=dev, dtype=grad_dtype) for _ in self.srcs]
            self.tail = e._g_flat[G * n * d:]  # [g_bias | extras]: all-reduced whole
        self.red_ev = None    # completion of this chunk's gradient reduction (current step)
        self.gath_ev = None   # completion of this chunk's shadow all-gather (ZeRO-1)


class GraphedDataParallel:
    def __init__(self, engines: Sequence, info: DistInfo, comm, source, mode: str = "dp",
                 grad_dtype: torch.dtype = torch.float32, count_every: int = 8, sync_params: bool = True,
                 capture: Optional[bool] = None):
        if mode not in ("dp", "zero1"):
            raise ValueError(f"mode must be 'dp' or 'zero1', got {mode!r}")
        self.info, self.comm, self.source, self.mode = info, comm, source, mode
        # capture=False: run the group's kernels and collectives eagerly (the same _steps sequence);
        # the default follows the communicator (a host-staged gloo comm cannot be captured)
        self.capture = getattr(comm, "capturable", True) if capture is None else bool(capture)
        self.chunks = [_Chunk(e, mode, info, grad_dtype) for e in engines]
        e0 = engines[0]
        self.B, self.d, self.device = e0.batch_size, e0.d, e0.device
        for e in engines:
            if e.batch_size != self.B or e.d != self.d:
                raise ValueError("every chunk engine must take the same [B, d] batch")
            e.grad_scale = 1.0 / max(1, info.world_size)
        self.x = torch.empty(self.B, self.d, device=self.device, dtype=torch.bfloat16)
        self._xs = None  # [s, B, d]: a group's batches, fetched in one launch at the group's start
        self.count_every = count_every
        self._graphs: Dict[tuple, torch.cuda.CUDAGraph] = {}
        if sync_params and info.world_size > 1:  # identical initial parameters: rank 0's
            for e in engines:
                for t in e.params.values():
                    comm.broadcast(t)
                e.refresh_shadows()
            torch.cuda.synchronize(self.device)

    # ------------------------------------------------------------------ one step (captured)
    def _compute(self, c: _Chunk, count: bool, x: torch.Tensor):
        e = c.engine
        e._counted = count
        xp = e.prepare(x)
        e.forward(xp, count)
        # both weight gradients in ONE grouped launch (the chunk's reduction waits for all of them
        # anyway), then the bias gradient into the flat buffer
        e.backward_weights(xp)
        e._reduce_bias_grad()

    def _reduce(self, c: _Chunk):
        e = c.engine
        if self.mode == "dp":
            c.red_ev = self.comm.all_reduce(e.grad_all, overlap=True)
            return
        evs = []
        if c.lowp:  # bf16 transport, fp32 accumulation on the row owner: every send buffer first, ...
            for i, src in enumerate(c.srcs):
                c.send[i].copy_(src.view(-1))
        # ... then the chunk's collectives back to back on ONE fork of the comm stream (RcclComm._run:
        # consecutive forks lose the next node's dependency under HIP graph capture)
        for i, (src, dst) in enumerate(zip(c.srcs, c.shards)):
            if c.lowp:
                evs.append(self.comm.all_to_all(c.recv[i], c.send[i], overlap=True, fork=not evs))
            elif c.world > 1:
                evs.append(self.comm.reduce_scatter(dst.view(-1), src.view(-1), overlap=True, fork=not evs))
        evs.append(self.comm.all_reduce(c.tail, overlap=True, fork=not evs))
        c.red_ev = evs

    def _wait(self, evs):
        if evs is None:
            return
        cur = torch.cuda.current_stream(self.device)
        for ev in (evs if isinstance(evs, list) else [evs]):
            if ev is not None:
                cur.wait_event(ev)

    def _update(self, c: _Chunk, gather=None):
        """The chunk's update after its reduction; ``gather`` (fused tail only): also copy the NEXT
        step's batch into the engines' input (see ``_steps``)."""
        e = c.engine
        self._wait(c.red_ev)
        c.red_ev = None
        if self.mode == "dp":
            if e._tail_ok:
                # the fused step tail (row Adam + losses + bias Adam, one launch) on the all-reduced
                # gradients: the bias gradient arrives reduced and scaled ([G, 1, n], gscale 1)
                adam_ops.step_tail(e._adam_sets(), e.lr, *e.betas, e.eps, e.step_dev, e.params[e._bkey],
                                   e.m[e._bkey], e.v[e._bkey], e.g_bias, e.enc_part, e.dec_part, e.l1,
                                   e.bias_decay, e.out, e.batch_size, 1.0, e._bsq, e._ticket,
                                   cnt_part=e.cnt_part if e._counted else None,
                                   feat_count=e.feature_counts if e._counted else None, live=e.nactive,
                                   gather=gather)
            else:
                e.adam_rows_all()
                e._bias_loss(update=True, reduced=True)
            return
        G, n, d = e.n_models, e.n, e.d
        lo, hi = c.lo, c.hi
        if c.world == 1:  # one rank: the shard is the whole gradient
            grads = c.srcs
        else:
            if c.lowp:
                for i, dst in enumerate(c.shards):
                    torch.sum(c.recv[i].view(c.world, -1), dim=0, dtype=torch.float32, out=dst.view(-1))
            grads = c.shards
        rows = lambda t: t.view(G * n, d)[lo:hi]  # noqa: E731
        g = [gg.view(-1, d) if c.world == 1 else gg for gg in grads]
        if e.kind == "untied":
            sets = [dict(p=rows(e.params["decoder"]), g=rows(g[0]) if c.world == 1 else g[0], m=rows(e.m["decoder"]),
                         v=rows(e.v["decoder"]), shadow=rows(e.dec_shadow), norms=e.norms.view(-1)[lo:hi], norm=True),
                    dict(p=rows(e.params["encoder"]), g=rows(g[1]) if c.world == 1 else g[1], m=rows(e.m["encoder"]),
                         v=rows(e.v["encoder"]), shadow=rows(e.enc_shadow), norms=None, norm=False)]
        else:
            sets = [dict(p=rows(e.params["encoder"]), g=rows(g[0]) if c.world == 1 else g[0], m=rows(e.m["encoder"]),
                         v=rows(e.v["encoder"]), shadow=rows(e.enc_shadow), norms=e.norms.view(-1)[lo:hi], norm=True)]
        if e._tail_ok:
            # the fused step tail on the owned rows (row Adam) + every model's losses and bias Adam
            # (the bias gradient arrives all-reduced and scaled)
            adam_ops.step_tail(sets, e.lr, *e.betas, e.eps, e.step_dev, e.params[e._bkey], e.m[e._bkey],
                               e.v[e._bkey], e.g_bias, e.enc_part, e.dec_part, e.l1, e.bias_decay, e.out,
                               e.batch_size, 1.0, e._bsq, e._ticket, cnt_part=e.cnt_part if e._counted else None,
                               feat_count=e.feature_counts if e._counted else None, row0=lo, gather=gather,
                               live=e.nactive)
        else:
            adam_ops.adam_rows(sets, e.lr, e.step_count + 1, *e.betas, e.eps, rows_per_model=n,
                               step_dev=e.step_dev, row0=lo, live=e.nactive)
            e._bias_loss(update=True, reduced=True)
        if c.world > 1:  # every rank's updated shadows (and norms) for the chunk's next compute
            evs = []
            for sh in ([e.dec_shadow] if e.kind == "untied" else []) + [e.enc_shadow]:
                flat = sh.view(-1)
                evs.append(self.comm.all_gather(flat, flat[lo * d:hi * d], overlap=True, fork=not evs))
            evs.append(self.comm.all_gather(e.norms.view(-1), e.norms.view(-1)[lo:hi], overlap=True, fork=False))
            c.gath_ev = evs

    def _steps(self, pattern: Sequence[bool]):
        """The kernels (and collectives) of ``len(pattern)`` steps; capture target."""
        e0 = self.chunks[0].engine
        K = len(self.chunks)
        s = len(pattern)
        prev: Optional[_Chunk] = None
        # The engines read every step's batch from self.x.  With a source, this rank's rows of all the
        # group's steps are fetched at its start in ONE launch (xs); step 0's batch is copied into x,
        # and the fused tail of the update that runs right before step i's first compute copies xs[i]
        # (through an identity index from the group's first step), so each encoder reads a batch
        # written just before it (L2 / MALL-hot, as in the single-GPU step).
        feed = None
        if self.source is not None:
            xs = self._xs_buffer(s)[:s]
            self.source.gather_steps(xs, e0.step_dev)
            if all(c.engine._tail_ok for c in self.chunks):
                self._ep0.copy_(e0.step_dev)
                feed = (self._xs.view(-1, self.d), self._ident, self._ep0, self.x)
            self.x.copy_(xs[0])
        for i, count in enumerate(pattern):
            if prev is not None and K == 1:  # one chunk: its update precedes its next compute
                self._update(prev, gather=feed)
                prev = None
            if self.source is not None and feed is None and i > 0:
                self.x.copy_(xs[i])
            for ci, c in enumerate(self.chunks):
                if c.gath_ev is not None:  # ZeRO-1: this chunk's shadows from the last update
                    self._wait(c.gath_ev)
                    c.gath_ev = None
                self._compute(c, count, self.x)
                self._reduce(c)
                if prev is not None:
                    # (K > 1: the update in the last chunk's slot is the one right before step i+1)
                    last = K > 1 and ci == K - 1 and i + 1 < s
                    self._update(prev, gather=feed if last else None)
                prev = c
        self._update(prev)
        for c in self.chunks:  # every side-stream op joins the capture before it ends
            self._wait(c.gath_ev)
            c.gath_ev = None
        self.comm.join()

    def _xs_buffer(self, s: int):
        if self._xs is None or self._xs.shape[0] < s:
            self._xs = torch.empty(s, self.B, self.d, device=self.device, dtype=torch.bfloat16)
            self._ident = torch.arange(s * self.B, device=self.device, dtype=torch.int64)
            self._ep0 = torch.zeros(1, device=self.device, dtype=torch.int32)
            self._graphs = {}  # captured on the old buffer
        return self._xs

    def _exec(self, pattern):
        """Replay the group's graph (captured on first use), or run its steps eagerly."""
        if self.capture:
            self._graph(pattern).replay()
            return
        if self.source is not None:
            self._xs_buffer(len(pattern))
        self._steps(tuple(bool(c) for c in pattern))

    def _graph(self, pattern):
        key = tuple(bool(c) for c in pattern)
        if self.source is not None:
            self._xs_buffer(len(key))
        g = self._graphs.get(key)
        if g is None:
            torch.cuda.synchronize(self.device)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                self._steps(key)
            from ..ops import _lib

            _lib.upload_graph(g, self.device)
            self._graphs[key] = g
        return g

    # ------------------------------------------------------------------ API
    def prime(self, patterns: Sequence[Sequence[bool]]):
        """Capture + upload (nothing runs) every group graph later replays use."""
        if self.source is not None:
            self._xs_buffer(max([1] + [len(p) for p in patterns]))
        for c in self.chunks:
            c.engine._tail_ready()
        for p in patterns:
            if self.capture:
                self._graph(p)
        e0 = self.chunks[0].engine
        if self.source is not None:
            self.source.prepare(e0.step_count, max([1] + [len(p) for p in patterns]))

    def run(self, steps: int, pattern: Optional[Sequence[bool]] = None):
        """``steps`` data-parallel optimizer steps as ONE graph replay."""
        e0 = self.chunks[0].engine
        if pattern is None:
            pattern = [i % self.count_every == 0 for i in range(int(steps))]
        pattern = tuple(bool(c) and e0.track_feature_counts for c in pattern)
        if self.source is None and len(pattern) != 1:
            raise ValueError("without a batch source every replay is one step on self.x (step_batch)")
        if self.source is not None:
            self.source.prepare(e0.step_count, len(pattern))
        for c in self.chunks:
            c.engine._tail_ready()
        self._exec(pattern)
        for c in self.chunks:
            for count in pattern:
                c.engine._counted = count
                c.engine._host_step()
        return [c.engine.out for c in self.chunks]

    def step_batch(self, x_local: torch.Tensor, count: Optional[bool] = None):
        """One step on this rank's rows ``x_local`` [B, d] (no in-graph source: EnsembleTrainer)."""
        self.x.copy_(x_local.to(self.device, torch.bfloat16))
        e0 = self.chunks[0].engine
        if count is None:
            count = e0._counting()
        return self.run(1, [count])

    def gather_masters(self):
        """ZeRO-1: every rank's fp32 masters and moments complete (exports / checkpoints)."""
        if self.mode != "zero1" or self.info.world_size <= 1:
            return
        for c in self.chunks:
            e = c.engine
            d = e.d
            keys = ["decoder", "encoder"] if e.kind == "untied" else ["encoder"]
            for store in (e.params, e.m, e.v):
                for k in keys:
                    flat = store[k].view(-1)
                    self.comm.all_gather(flat, flat[c.lo * d:c.hi * d])
        torch.cuda.synchronize(self.device)

    def to_learned_dicts(self, device="cpu") -> List:
        self.gather_masters()
        return [ld for c in self.chunks for ld in c.engine.to_learned_dicts(device)]


class GraphedEnsembleSharded:
    """Ensemble-axis sharding (``parallel/ensemble_shard.py``) with the batch all-gathers INSIDE the
    multi-step HIP graph.

    Per group of s steps, one graph holds: ONE gather kernel writing this rank's rows of all s steps
    straight into its slots of the s global batches (``RingGraphSource.gather_into_global``, device
    step counter), s in-place all-gathers on the communicator's stream (``parallel/rccl.py``), and the
    s steps of the rank's models, step k waiting on exactly gather k's event -- so gather k+1.. run
    under step k's GEMMs and no collective is issued from the host.  Per model the update is the
    data-parallel one on the N B global rows, as in ``EnsembleSharded``.  Reference: the sweep
    sharding of ``cluster_runs.py:100-157`` / DDP of ``experiments/huge_batch_size.py:259-345``.
    """

    def __init__(self, es, comm, source, capture: Optional[bool] = None):
        e = es.engine
        if not hasattr(e, "_step_kernels") or not hasattr(e, "step_dev"):
            raise NotImplementedError("graphed ensemble sharding needs the fused engine")
        if getattr(source, "world", 1) != es.info.world_size or getattr(source, "rank", 0) != es.info.rank:
            raise ValueError("the source must be this rank's shard (ring.graph_source(B, rank, world))")
        self.es, self.comm, self.source, self.engine = es, comm, source, e
        # capture=False: the same _steps sequence run eagerly (host-staged gloo comm: not capturable)
        self.capture = getattr(comm, "capturable", True) if capture is None else bool(capture)
        self.B, self.N = es.B, max(1, es.info.world_size)
        self.device = e.device
        self._glob = None
        self._graphs: Dict[tuple, torch.cuda.CUDAGraph] = {}

    def _buffers(self, s: int):
        if self._glob is None or self._glob.shape[0] < s:
            NB = self.N * self.B
            self._glob = torch.zeros(s, NB, self.es.d, device=self.device, dtype=torch.bfloat16)
            # the engine's input and the tail-gather plumbing: step k's fused tail copies global batch
            # k+1 into it (rows (t + 1 - ep0) NB + r of the group buffer through an identity index),
            # so each step's encoder reads a batch written just before it -- as the single-GPU step
            self._x = torch.empty(NB, self.es.d, device=self.device, dtype=torch.bfloat16)
            self._ident = torch.arange(s * NB, device=self.device, dtype=torch.int64)
            self._ep0 = torch.zeros(1, device=self.device, dtype=torch.int32)
            self._graphs = {}  # captured on the old buffers
        return self._glob

    def _steps(self, pattern):
        e = self.engine
        s = len(pattern)
        glob = self._buffers(s)[:s]
        self.source.gather_into_global(glob, e.step_dev)
        B, r = self.B, self.es.info.rank
        cur = torch.cuda.current_stream(self.device)
        tail = bool(e._tail_ok)
        if tail:
            self._ep0.copy_(e.step_dev)  # the group's first step: the tail's index base
            flat = self._glob.view(-1, self.es.d)
        # the s all-gathers on ONE fork of the comm stream (RcclComm._run: with one fork per collective,
        # HIP graph capture dropped the dependency of the next node -- this ep0 copy, read by every
        # tail -- on the gather above, and group replays raced; profiles/r6/graph_capture/)
        evs = [self.comm.all_gather(glob[k], glob[k][r * B:(r + 1) * B], overlap=True, fork=k == 0) for k in range(s)]
        for k, count in enumerate(pattern):
            if k == 0 or not tail:
                if evs[k] is not None:
                    cur.wait_event(evs[k])
                self._x.copy_(glob[k])
            nxt = tail and k + 1 < s
            # the tail of step k reads global batch k+1: only the update waits for that gather
            wait = (lambda ev=evs[k + 1]: cur.wait_event(ev)) if nxt and evs[k + 1] is not None else None
            e._counted = count
            e._step_kernels(self._x, count, gather=(flat, self._ident, self._ep0, self._x) if nxt else None,
                            before_update=wait)
        self.comm.join()

    def _graph(self, pattern):
        key = tuple(bool(c) for c in pattern)
        self._buffers(len(key))
        g = self._graphs.get(key)
        if g is None:
            torch.cuda.synchronize(self.device)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                self._steps(key)
            from ..ops import _lib

            _lib.upload_graph(g, self.device)
            self._graphs[key] = g
        return g

    def prime(self, patterns):
        """Capture + upload (nothing runs) every group graph later replays use."""
        e = self.engine
        self._buffers(max([1] + [len(p) for p in patterns]))
        e._tail_ready()
        for p in patterns:
            if self.capture:
                self._graph(tuple(bool(c) and e.track_feature_counts for c in p))
        self.source.prepare(e.step_count, max([1] + [len(p) for p in patterns]))

    def run(self, steps: int, pattern=None):
        """``steps`` ensemble-sharded optimizer steps as ONE graph replay."""
        e = self.engine
        if pattern is None:
            pattern = [i == 0 for i in range(int(steps))]
        pattern = tuple(bool(c) and e.track_feature_counts for c in pattern)
        if len(pattern) != int(steps):
            raise ValueError("one counting flag per step")
        e._tail_ready()
        self.source.prepare(e.step_count, len(pattern))
        if self.capture:
            self._graph(pattern).replay()
        else:
            self._buffers(len(pattern))
            self._steps(pattern)
        for count in pattern:
            e._counted = count
            e._host_step()
        return e.out
