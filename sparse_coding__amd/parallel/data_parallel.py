"""Data-parallel ensemble training with overlapped gradient all-reduce.

Reference: the DDP experiment ``experiments/huge_batch_size.py:259-345`` (gloo,
implicit bucketed all-reduce in ``backward``).  Here every rank holds the full
ensemble, consumes its own batch shard, and the gradients are summed with
explicit collectives (RCCL over xGMI on MI355X; gloo on CPU).

Overlap schedule for the fused engine (one step, compute stream on the left,
RCCL stream on the right)::

    enc / dec / code-grad GEMMs
    dW_hat = c^T R            -> all_reduce(dW_hat)           (async)
    dW_e = dpre^T x, db       |  ... dW_hat in flight ...
                              -> all_reduce([dW_e | db])      (async, one flat buffer)
    wait(dW_hat); Adam(decoder)  ... [dW_e | db] in flight ...
    wait([dW_e | db]); Adam(encoder); bias Adam + losses

Each collective is issued with ``async_op=True`` so ProcessGroupNCCL orders it
after the producing kernel and the compute stream only waits at the consumer.
Gradients are pre-scaled by 1/world_size inside the GEMM epilogue (alpha), so a
SUM all-reduce yields the global-batch mean gradient with no extra pass.
"""

from __future__ import annotations

import torch
import torch.distributed as dist
from torch.utils import _pytree as pytree

from .dist import DistInfo


class DataParallelFused:
    """Wraps a ``FusedSAEEnsemble``; identical parameters on every rank after each step."""

    def __init__(self, engine, info: DistInfo, grad_dtype: torch.dtype = torch.float32):
        self.engine = engine
        self.info = info
        self.grad_dtype = grad_dtype
        engine.grad_scale = 1.0 / info.world_size
        if info.enabled:
            engine.fuse_adam = False  # gradients are all-reduced before the (separate) Adam kernels
            self.sync_params()

    def sync_params(self):
        """Broadcast rank 0's parameters (identical init on every rank)."""
        e = self.engine
        for t in e.params.values():
            dist.broadcast(t, src=0)
        e.refresh_shadows()

    def _all_reduce(self, t):
        if self.grad_dtype == torch.float32:
            return dist.all_reduce(t, async_op=True), None
        buf = t.to(self.grad_dtype)
        return dist.all_reduce(buf, async_op=True), (buf, t)

    @staticmethod
    def _finish(work, pair):
        work.wait()
        if pair is not None:
            pair[1].copy_(pair[0])

    def step_batch(self, batch):
        e = self.engine
        x = e._x_bf16(batch)
        if not self.info.enabled:
            return e.step_batch(x)
        e.forward(x)
        e.wgrad_first(x)
        first = e.g_dec if e.kind == "untied" else e._g_flat
        w1 = self._all_reduce(first)
        e.wgrad_second(x)
        w2 = self._all_reduce(e._g_flat) if e.kind == "untied" else None
        self._finish(*w1)
        e.adam_first()
        if w2 is not None:
            self._finish(*w2)
        e.adam_second(reduced_bias=True)
        return e.out

    def mean_losses(self):
        out = self.engine.out.clone()
        if self.info.enabled:
            dist.all_reduce(out)
            out /= self.info.world_size
        return out


class DataParallelEnsemble:
    """Data parallelism for the eager ``FunctionalEnsemble`` (any signature, CPU/gloo capable)."""

    def __init__(self, ensemble, info: DistInfo, bucket_bytes: int = 64 << 20):
        self.ensemble = ensemble
        self.info = info
        self.bucket_bytes = bucket_bytes
        if info.enabled:
            for t in pytree.tree_leaves(ensemble.params):
                dist.broadcast(t.data, src=0)

    def _reduce(self, grads):
        leaves = pytree.tree_leaves(grads)
        # bucket the leaves into flat buffers of ~bucket_bytes and reduce each asynchronously
        buckets, cur, size = [], [], 0
        for t in leaves:
            cur.append(t)
            size += t.numel() * t.element_size()
            if size >= self.bucket_bytes:
                buckets.append(cur)
                cur, size = [], 0
        if cur:
            buckets.append(cur)
        works = []
        for b in buckets:
            flat = torch.cat([t.reshape(-1) for t in b])
            works.append((dist.all_reduce(flat, async_op=True), flat, b))
        for w, flat, b in works:
            w.wait()
            flat /= self.info.world_size
            off = 0
            for t in b:
                t.copy_(flat[off:off + t.numel()].view_as(t))
                off += t.numel()

    def step_batch(self, batch):
        grads, (loss, aux) = self.ensemble.compute_grads(batch)
        if self.info.enabled:
            self._reduce(grads)
        self.ensemble.apply_grads(grads)
        return loss, aux
