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


def _check_kind(engine):
    # threshold / learned-centering SAEs carry their scale / centering gradient sources in the
    # same flat buffer (engine._g_flat), so every fused kind reduces with the same collectives
    if getattr(engine, "kind", None) not in ("untied", "tied", "reverse", "threshold"):
        raise NotImplementedError(f"data-parallel fused training of kind {getattr(engine, 'kind', None)}")


class DataParallelFused:
    """Wraps a ``FusedSAEEnsemble``; identical parameters on every rank after each step."""

    def __init__(self, engine, info: DistInfo, grad_dtype: torch.dtype = torch.float32):
        _check_kind(engine)
        self.engine = engine
        self.info = info
        self.grad_dtype = grad_dtype
        engine.grad_scale = 1.0 / info.world_size
        if info.enabled:
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
        x = e.prepare(x)
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


# ----------------------------------------------------------------------------- model-chunk pipelining
class FusedChunk:
    """Adapter: one ``FusedSAEEnsemble`` (a chunk of the ensemble's models) as a pipeline stage.

    ``graph=True``: the chunk's compute (forward + weight gradients) and its update (Adam, bias
    Adam, losses) each replay from a HIP graph captured on first use; the all-reduce between
    them is issued from the host (one process launches ~4 graphs per step instead of ~10
    kernels per chunk).  ``x_static``: the persistent input buffer the batch arrives in."""

    def __init__(self, engine, graph: bool = False, x_static=None):
        _check_kind(engine)
        self.engine = engine
        self.graph = graph
        self.x_static = x_static
        self._graphs = {}

    def set_grad_scale(self, s: float):
        self.engine.grad_scale = s

    def params(self):
        return list(self.engine.params.values())

    def after_param_sync(self):
        self.engine.refresh_shadows()

    def compute_grads(self, x):
        from .zero import graphed_region

        e = self.engine
        if self.graph:
            if self.x_static is None:
                self.x_static = torch.empty(e.batch_size, e.d, device=e.device, dtype=torch.bfloat16)
            if x is not self.x_static:
                self.x_static.copy_(x)
            x = self.x_static
        else:
            x = e._x_bf16(x)
        count = e._counting()
        e._counted = count

        def run():
            xp = e.prepare(x)
            e.forward(xp, count)
            e.wgrad_first(xp)
            e.wgrad_second(xp, reduce_bias=True)  # pre-scaled by 1/world: SUM all-reduce = mean

        graphed_region(self, "grads", run)
        return e.grad_all

    def apply_update(self, grad_flat):
        from .zero import graphed_region

        e = self.engine

        def run():
            if e.kind == "threshold" or e.learned_center:
                e._threshold_extra_adam(reduced=True)
            e.adam_rows_all()
            e._bias_loss(update=True, reduced=True)

        graphed_region(self, "update", run)
        e._host_step()
        return e.out


class EagerChunk:
    """Adapter: one eager ``FunctionalEnsemble`` chunk (CPU / gloo tests, unfused signatures)."""

    def __init__(self, ensemble):
        self.ens = ensemble
        self.scale = 1.0
        self._grads = None
        self._spec = None
        self.last = None

    def set_grad_scale(self, s: float):
        self.scale = s

    def params(self):
        return [t.data for t in pytree.tree_leaves(self.ens.params)]

    def after_param_sync(self):
        pass

    def compute_grads(self, x):
        grads, (loss, aux) = self.ens.compute_grads(x)
        self.last = loss
        leaves, self._spec = pytree.tree_flatten(grads)
        self._shapes = [t.shape for t in leaves]
        return torch.cat([t.reshape(-1) for t in leaves]) * self.scale

    def apply_update(self, grad_flat):
        leaves, off = [], 0
        for shp in self._shapes:
            k = int(torch.Size(shp).numel())
            leaves.append(grad_flat[off:off + k].view(shp))
            off += k
        self.ens.apply_grads(pytree.tree_unflatten(leaves, self._spec))
        return self.last


class ChunkedDataParallel:
    """Data parallelism with the ensemble split into model chunks whose gradient
    all-reduce overlaps the NEXT chunk's compute.

    The models of an ensemble are independent, so chunk k's update needs only chunk
    k's reduced gradients.  Per step (compute stream | RCCL stream)::

        fwd+bwd chunk 0            -> AR(grads 0)
        fwd+bwd chunk 1            |  AR 0 in flight      -> AR(grads 1)
        wait AR 0; Adam chunk 0    |  AR 1 in flight
        fwd+bwd chunk 2            |                      -> AR(grads 2)
        wait AR 1; Adam chunk 1    ...

    Only the last chunk's all-reduce is exposed (a 1/K share of the traffic), instead of
    the whole ensemble's gradients as in a reduce-after-backward step.  Every rank issues
    the same collectives in the same order; gradients are pre-scaled by 1/world so a SUM
    all-reduce yields the global mean.  Numerically identical to training each chunk on
    the global batch (the reference's DDP semantics, huge_batch_size.py:259-345).
    """

    def __init__(self, chunks, info: DistInfo, grad_dtype: torch.dtype = torch.float32,
                 cross_step: bool = False):
        self.chunks = list(chunks)
        self.info = info
        self.grad_dtype = grad_dtype
        # cross_step: the LAST chunk's all-reduce is left in flight at the end of a step and
        # completed (wait + Adam) only after the next step's first chunk has computed, so
        # it overlaps the next step's encoder GEMM instead of being exposed.  Call
        # ``flush()`` before reading parameters.
        self.cross_step = cross_step and len(self.chunks) > 1
        self._carry = None
        for c in self.chunks:
            c.set_grad_scale(1.0 / info.world_size)
        if info.enabled:
            for c in self.chunks:
                for t in c.params():
                    dist.broadcast(t, src=0)
                c.after_param_sync()

    def _reduce_async(self, flat):
        if not dist.is_initialized() or self.info.world_size <= 1:  # one rank: the sum is the gradient
            return None, flat
        if self.grad_dtype == torch.float32 or flat.dtype == self.grad_dtype:
            return dist.all_reduce(flat, async_op=True), flat
        buf = flat.to(self.grad_dtype)
        return (dist.all_reduce(buf, async_op=True), (buf, flat))

    @staticmethod
    def _finish(work, payload):
        if work is not None:
            work.wait()
        if isinstance(payload, tuple):
            payload[1].copy_(payload[0])
            return payload[1]
        return payload

    def _reduce(self, c, flat):
        # chunks with their own collective pattern (ZeRO-1: reduce-scatter + all-reduce of the
        # bias) return a pending handle; the default is one all-reduce of the flat gradient
        h = c.reduce_async() if hasattr(c, "reduce_async") else self._reduce_async(flat)
        if serialized():  # race debugging (utils.debug.serialize_streams): no overlap at all
            torch.cuda.synchronize() if torch.cuda.is_available() else None
            if hasattr(h, "wait") and not isinstance(h, tuple):
                h.wait()
            elif h[0] is not None:
                h[0].wait()
        return h

    def _complete(self, j, handle):
        c = self.chunks[j]
        if hasattr(handle, "wait") and not isinstance(handle, tuple):
            handle.wait()
            return c.apply_update(None)
        return c.apply_update(self._finish(*handle))

    def step_batch(self, x):
        outs = [None] * len(self.chunks)
        pending = []
        last = len(self.chunks) - 1
        for k, c in enumerate(self.chunks):
            if k == last and self._carry is not None:
                raise RuntimeError("unreachable: carried update must complete before its chunk computes")
            flat = c.compute_grads(x)
            if k == 0 and self._carry is not None:
                # the previous step's last chunk: its reduction overlapped this chunk's compute
                j, h = self._carry
                self._carry = None
                outs[j] = self._complete(j, h)
            pending.append((k, self._reduce(c, flat)))
            if len(pending) > 1:  # previous chunk's reduction had this chunk's compute to hide behind
                j, h = pending.pop(0)
                outs[j] = self._complete(j, h)
        if self.cross_step:
            self._carry = pending.pop()  # completes during the next step's first chunk
        for j, h in pending:
            outs[j] = self._complete(j, h)
        return outs

    def flush(self):
        """Complete a carried (cross-step) update; parameters are then current."""
        if self._carry is not None:
            j, h = self._carry
            self._carry = None
            return self._complete(j, h)
        return None


def serialized() -> bool:
    """``SC_SERIALIZE_STREAMS=1`` (``utils.debug.serialize_streams``): every collective completes
    before the next kernel is issued -- overlap-induced races show up as result differences."""
    import os

    return os.environ.get("SC_SERIALIZE_STREAMS", "0") not in ("", "0")


def split_models(models, n_chunks: int):
    """Contiguous, near-equal chunks of an ensemble's model list."""
    n_chunks = max(1, min(n_chunks, len(models)))
    per = -(-len(models) // n_chunks)
    return [models[i:i + per] for i in range(0, len(models), per)]
