"""Ensemble-axis sharding with a global batch: the multi-GPU mode built for xGMI.

The reference trains an L1 sweep as one ensemble per device (sweep sharding,
``big_sweep_experiments.py:49,66``; ``cluster_runs.py:100-157``) and has a separate
DDP experiment whose gradient all-reduce moves the whole parameter set every step
(``experiments/huge_batch_size.py:259-345``).  For an SAE ensemble the gradient is
as large as the parameters -- 2 x G x n x d fp32, 67 MB for 8 models at d=512, n=2048
-- while the batch that produces it is tiny (B x d bf16 = 2 MB).  On MI355X the
per-GPU xGMI bandwidth a ring collective can use is a few links of ~64-76 GB/s per
direction (one link between two GPUs), so a gradient all-reduce costs as much as or
more than the 0.34 ms step it belongs to.

This mode moves the *batch* instead of the gradients.  With N ranks and G models
(G % N == 0):

* rank r owns models ``[r G/N, (r+1) G/N)`` -- their fp32 masters, Adam moments and
  bf16 shadows live only there (1/N of the parameter memory and of the Adam traffic);
* every rank samples its own B rows (the DistributedSampler shard of the global
  permutation) and one ``all_gather_into_tensor`` (RCCL) assembles the global batch
  [N B, d] on every rank (2 MB per rank at d=512, B=2048);
* each rank runs the full fused step for its models on the global batch.

Per model this is *exactly* the data-parallel update on the global batch of N B rows
(the gradient is the mean over the same N B rows); the FLOPs per GPU equal the
single-GPU step's (G/N models x N B rows), so the scaling is weak.  The gather for
step t+1 is issued before step t's kernels and overlaps them (RCCL's own stream),
so the only communication on the critical path is the first step's gather.

``EnsembleSharded`` is engine-agnostic: ``FusedSAEEnsemble`` on MI355X (one HIP
graph per step), ``AnalyticSAEEnsemble`` on the CPU (gloo tests).
"""

from __future__ import annotations

from typing import Callable, List, Optional, Sequence

import torch
import torch.distributed as dist

from .dist import DistInfo


def shard_range(n_models: int, info: DistInfo):
    """Models owned by this rank (contiguous block); requires n_models % world == 0."""
    N = info.world_size
    if n_models % N:
        raise ValueError(f"ensemble sharding needs n_models % world_size == 0 (got {n_models} models, {N} ranks)")
    per = n_models // N
    return info.rank * per, (info.rank + 1) * per


class EnsembleSharded:
    """Each rank trains its block of the ensemble on the all-gathered global batch.

    ``engine_factory(models, batch_size)`` builds the per-rank engine (it must expose
    ``step_batch(x)``, ``params`` (dict of stacked [G_local, ...] tensors) and
    ``unstack(device)`` / ``sig``).  ``batch_per_rank`` rows are sampled per rank per
    step; the engine sees ``world_size * batch_per_rank`` rows.
    """

    def __init__(self, models: Sequence, engine_factory: Callable, info: DistInfo, batch_per_rank: int,
                 d: int, dtype: torch.dtype = torch.bfloat16):
        self.info = info
        self.n_models = len(models)
        self.lo, self.hi = shard_range(self.n_models, info)
        self.B = int(batch_per_rank)
        self.d = d
        self.global_batch = self.B * info.world_size
        self.engine = engine_factory(list(models[self.lo:self.hi]), self.global_batch)
        dev = info.device
        # double-buffered global batch: step t reads one while step t+1's gather fills the other
        self.gbuf = [torch.empty(self.global_batch, d, device=dev, dtype=dtype) for _ in range(2)]
        self.lbuf = [torch.empty(self.B, d, device=dev, dtype=dtype) for _ in range(2)]
        self._cur = 0
        self._pending = None  # (buffer index, work) of the gather in flight

    def enable_graph(self):
        """Fused engine: one HIP graph per step, captured on each of the two gather buffers
        (the gathered batch is consumed in place, no copy into the engine's input)."""
        self.engine.enable_graph()
        for t in self.gbuf:
            self.engine.add_static_input(t)
        self.engine._capture()  # now, before any collective is in flight
        return self

    # ------------------------------------------------------------------ batch assembly
    def _gather(self, local: torch.Tensor, i: Optional[int], async_op: bool, out: Optional[torch.Tensor] = None):
        out = self.gbuf[i] if out is None else out
        if not dist.is_initialized():
            out.copy_(local)
            return None
        if self.info.backend == "gloo":  # gloo: list all_gather through host memory (tests, rehearsals)
            host = local.detach().cpu()
            parts = [torch.empty_like(host) for _ in range(self.info.world_size)]
            dist.all_gather(parts, host)
            out.copy_(torch.cat(parts))
            return None
        return dist.all_gather_into_tensor(out, local.contiguous(), async_op=async_op)

    def step_batch(self, local: torch.Tensor):
        """One step on this rank's ``local`` rows [B, d] (gathered synchronously)."""
        i = self._cur
        self.lbuf[i].copy_(local)
        w = self._gather(self.lbuf[i], i, async_op=False)
        if w is not None and hasattr(w, "wait"):
            w.wait()
        self._cur = 1 - i
        return self.engine.step_batch(self.gbuf[i])

    def step_sampled(self, sample: Callable[[torch.Tensor], torch.Tensor]):
        """Overlapped step: ``sample(out)`` writes this rank's next [B, d] rows into ``out``.
        The gather of step t+1's batch is issued before step t's kernels, so it runs on
        RCCL's stream while they execute."""
        if self._pending is None:  # first step: nothing prefetched yet
            i = self._cur
            sample(self.lbuf[i])
            self._pending = (i, self._gather(self.lbuf[i], i, async_op=True))
        i, work = self._pending
        if work is not None:
            work.wait()  # stream-ordered: compute waits for the gather, the host does not block
        nxt = 1 - i
        sample(self.lbuf[nxt])
        self._pending = (nxt, self._gather(self.lbuf[nxt], nxt, async_op=True))
        self._cur = nxt
        return self.engine.step_batch(self.gbuf[i])

    # ------------------------------------------------------------------ multi-step groups
    def _group_buffers(self, s: int):
        """Per parity: a send buffer [s_max B, d] (this rank's rows of a group's steps) and the
        gathered global batches [s_max, N B, d], one contiguous [N B, d] buffer per step."""
        have = getattr(self, "_gsend", None)
        if have is None or have[0].shape[0] < s * self.B:
            dev, dt = self.gbuf[0].device, self.gbuf[0].dtype
            self._gsend = [torch.empty(s * self.B, self.d, device=dev, dtype=dt) for _ in range(2)]
            self._gglob = [torch.zeros(s, self.global_batch, self.d, device=dev, dtype=dt) for _ in range(2)]
        return self._gsend, self._gglob

    def _issue_group(self, par: int, s: int, sample_steps):
        send, glob = self._group_buffers(s)
        sample_steps(send[par][: s * self.B], s)
        works = [self._gather(send[par][k * self.B:(k + 1) * self.B], None, async_op=True, out=glob[par][k])
                 for k in range(s)]
        return par, s, works

    def prime_groups(self, sizes: Sequence[int], pattern_fn):
        """Fused engine: capture + upload every multi-step graph ``run_groups`` will replay (both
        buffer parities), before any collective is in flight."""
        if not hasattr(self.engine, "prime_inputs"):
            return
        _, glob = self._group_buffers(max(sizes))
        for s in sorted(set(sizes)):
            for par in (0, 1):
                self.engine.prime_inputs([glob[par][k] for k in range(s)], pattern_fn(s))

    def run_groups(self, groups: Sequence[int], sample_steps, pattern_fn=None):
        """``sum(groups)`` steps as multi-step groups: per group ONE ``sample_steps(out, s)`` call (this
        rank's rows of the group's s steps, e.g. ``DeviceRing.sample_shard_steps``), s batch
        all-gathers on RCCL's stream, and ONE graph replay of the s steps (fused engine; other engines
        step each batch).  The next group's sample and gathers are issued before this group's replay,
        so they run under it; a replay waits (stream-ordered, no host sync) for its own gathers."""
        groups = [int(s) for s in groups if int(s) > 0]
        if not groups:
            return None
        pattern_fn = pattern_fn or (lambda s: [i == 0 for i in range(s)])
        self.flush()  # (a single-step prefetch of step_sampled would hold stale rows)
        self._group_buffers(max(groups))  # (re)allocated before anything is gathered into them
        par = self._gpar = getattr(self, "_gpar", 0)
        pend = self._issue_group(par, groups[0], sample_steps)
        out = None
        for k, s in enumerate(groups):
            p, _, works = pend
            for w in works:
                if w is not None:
                    w.wait()
            if k + 1 < len(groups):
                pend = self._issue_group(1 - p, groups[k + 1], sample_steps)
            glob = self._gglob[p]
            if hasattr(self.engine, "step_inputs"):
                out = self.engine.step_inputs([glob[p_k] for p_k in range(s)], pattern_fn(s))
            else:
                for i in range(s):
                    out = self.engine.step_batch(glob[i])
        self._gpar = 1 - pend[0]
        return out

    def flush(self):
        """Complete an outstanding prefetch (call before tearing the process group down)."""
        if self._pending is not None:
            _, work = self._pending
            if work is not None:
                work.wait()
            self._pending = None

    # ------------------------------------------------------------------ results
    def gather_params(self, keys: Optional[List[str]] = None) -> dict:
        """Stacked parameters of the WHOLE ensemble on every rank (all-gather of each key)."""
        p = self.engine.params
        keys = list(p) if keys is None else keys
        out = {}
        for k in keys:
            t = p[k].detach().contiguous()
            if not dist.is_initialized():
                out[k] = t.clone()
                continue
            dev = t.device
            if self.info.backend == "gloo":
                t = t.cpu()
            parts = [torch.empty_like(t) for _ in range(self.info.world_size)]
            dist.all_gather(parts, t)
            out[k] = torch.cat(parts).to(dev)
        return out

    def to_learned_dicts(self, models_meta: Sequence[dict], sig, device="cpu"):
        """LearnedDicts of all G models (collective: every rank must call it)."""
        full = self.gather_params()
        out = []
        for g in range(self.n_models):
            p = {k: v[g].to(device).clone() for k, v in full.items()}
            b = {k: (v.detach().to(device).clone() if torch.is_tensor(v) else v) for k, v in models_meta[g].items()}
            out.append(sig.to_learned_dict(p, b))
        return out
