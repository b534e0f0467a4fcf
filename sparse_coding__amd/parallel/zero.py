"""ZeRO-1 data parallelism for SAE ensembles: reduce-scatter -> sharded Adam -> all-gather.

Reference: the DDP experiment ``experiments/huge_batch_size.py:259-345`` (implicit all-reduce of
the full gradient in ``backward``, then every rank runs the full Adam).  Here each rank owns a
contiguous 1/N shard of the ensemble's dictionary ROWS (rows of [G * n, d], whole rows so the
decoder's row-norm Jacobian stays local), and per step:

    fwd + bwd GEMMs on the local batch          (every rank, all models)
    reduce_scatter(dW_hat)  -> owned rows        \\  fp32 (or bf16) sums of the local
    reduce_scatter(dW_e)    -> owned rows         |  gradients, pre-scaled by 1/N in the
    all_reduce([db | extras])                    /   GEMM epilogue (= global-batch mean)
    Adam on the owned rows only (1/N of the optimizer's HBM traffic)
    all_gather(bf16 shadows)                     -> every rank's GEMM operands for the next step

Per GPU and step this moves (N-1)/N x (gradient + shadow) bytes instead of the all-reduce's
2 (N-1)/N x gradient bytes (fp32 gradients: 100 vs 134 MB for the headline 8-model ensemble),
and Adam's ~500 MB of p/g/m/v traffic shrinks to 1/N.  Semantics are exactly data-parallel
Adam on the global batch: the fp32 masters and moments of a row live on its owner; the other
ranks' copies of those masters are stale until ``gather_masters()`` (called by exports).

``ZeroFusedChunk`` plugs the fused engine into ``ChunkedDataParallel`` (model-chunk pipeline:
chunk k's collectives overlap chunk k+1's compute) and optionally captures each chunk's
compute and update kernels as HIP graphs; ``ZeroEagerChunk`` is the same protocol over a flat
parameter vector for any eager ``FunctionalEnsemble`` signature (CPU / gloo tests).
"""

from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist
from torch.utils import _pytree as pytree

from .dist import DistInfo


def shard_range(total: int, rank: int, world: int):
    """[lo, hi) of ``total`` rows owned by ``rank`` (requires total % world == 0)."""
    if total % world:
        raise ValueError(f"{total} rows do not split evenly over {world} ranks")
    per = total // world
    return rank * per, (rank + 1) * per


def comm_bytes_per_step(mode: str, world: int, grad_bytes: int, shadow_bytes: int = 0, batch_bytes: int = 0) -> int:
    """Bytes each GPU sends per step (ring collectives) for the data-parallel modes: ``dp``
    all-reduce 2 (N-1)/N g; ``zero1`` reduce-scatter + all-gather (N-1)/N (g + s); ``es``
    (ensemble sharding) all-gather of the global batch (N-1)/N b (b = the gathered N B rows)."""
    f = (world - 1) / world
    if mode == "dp":
        return int(2 * f * grad_bytes)
    if mode == "zero1":
        return int(f * (grad_bytes + shadow_bytes))
    if mode == "es":
        return int(f * batch_bytes)
    raise ValueError(mode)


def _gloo_cuda(t) -> bool:
    """gloo moves CUDA tensors for all-reduce / broadcast only (tests with several ranks sharing
    one GPU): reduce-scatter and all-gather then go through an all-reduce."""
    return t.is_cuda and dist.get_backend() == "gloo"


def reduce_scatter_async(out, inp):
    """out = this rank's 1/N slice of sum_ranks(inp) (async handle or None when completed)."""
    if _gloo_cuda(inp):
        tmp = inp.clone()
        dist.all_reduce(tmp)
        r = dist.get_rank()
        out.copy_(tmp.view(dist.get_world_size(), -1)[r])
        return None
    return dist.reduce_scatter_tensor(out, inp, async_op=True)


def reduce_scatter_lowp(out, inp, send, recv):
    """out (fp32) = this rank's 1/N slice of sum_ranks(inp), moving ``send.dtype`` (bf16) over the
    links but accumulating in fp32 on the owner: every rank sends rank j's slice of its (rounded)
    gradient to j (all-to-all), and the owner sums the N received slices in fp32.  Same bytes per
    GPU as a bf16 reduce-scatter, (N-1)/N x g/2, without the ring's N-1 bf16 re-roundings of the
    partial sums.  Synchronous on the host only for gloo (CPU transport); returns a work handle or
    None, and a finisher that does the fp32 sum once the transfer completed."""
    world = dist.get_world_size()
    send.copy_(inp.view(-1))
    if send.is_cuda and dist.get_backend() == "gloo":  # gloo moves CPU tensors only for all-to-all
        s_cpu, r_cpu = send.cpu(), torch.empty(recv.shape, dtype=recv.dtype)
        dist.all_to_all_single(r_cpu, s_cpu)
        recv.copy_(r_cpu)
        work = None
    else:
        work = dist.all_to_all_single(recv, send, async_op=True)

    def finish():
        torch.sum(recv.view(world, -1), dim=0, dtype=torch.float32, out=out.view(-1))

    return work, finish


def all_gather_async(flat, lo, hi):
    """Every rank's [lo, hi) slice of ``flat`` (its own slice is current) into all ranks' ``flat``."""
    if _gloo_cuda(flat):
        tmp = torch.zeros_like(flat)
        tmp[lo:hi] = flat[lo:hi]
        dist.all_reduce(tmp)
        flat.copy_(tmp)
        return None
    return dist.all_gather_into_tensor(flat, flat[lo:hi], async_op=True)


def graphed_region(chunk, key, fn):
    """Run ``fn`` (kernel launches only) -- from a HIP graph captured on first use when
    ``chunk.graph`` is set; one graph per (key, feature-counting step or not)."""
    e = chunk.engine
    if not chunk.graph:
        fn()
        return
    count = e._counting()
    g = chunk._graphs.get((key, count))
    if g is None:
        torch.cuda.synchronize(e.device)
        g = torch.cuda.CUDAGraph()
        # thread_local: RCCL's watchdog thread may query events of in-flight collectives
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            fn()
        chunk._graphs[(key, count)] = g
    g.replay()


class _Pending:
    """Async collectives plus what to do once they completed."""

    def __init__(self):
        self.works = []
        self.after = []

    def add(self, work, after=None):
        if work is not None:
            self.works.append(work)
        if after is not None:
            self.after.append(after)

    def wait(self):
        for w in self.works:
            w.wait()
        for f in self.after:
            f()
        self.works, self.after = [], []


class ZeroFusedChunk:
    """One ``FusedSAEEnsemble`` (a chunk of the ensemble's models) under ZeRO-1.

    Row shards: rank r owns rows [lo, hi) of the flattened [G * n] dictionary rows (decoder and
    encoder alike).  ``graph=True`` replays the chunk's compute (forward + weight gradients)
    and update (shard Adam + bias Adam + losses) from HIP graphs; the collectives are issued
    from the host between the replays (RCCL orders them after the producing kernels)."""

    def __init__(self, engine, info: DistInfo, grad_dtype: torch.dtype = torch.float32, graph: bool = False,
                 x_static: Optional[torch.Tensor] = None):
        kind = getattr(engine, "kind", None)
        if kind not in ("untied", "tied") or engine.learned_center:
            raise NotImplementedError(f"ZeRO-1 fused training of kind {kind}")
        self.engine = e = engine
        self.info = info
        self.grad_dtype = grad_dtype
        G, n, d = e.n_models, e.n, e.d
        self.lo, self.hi = shard_range(G * n, info.rank, info.world_size)
        rows = self.hi - self.lo
        dev = e.device
        # one rank: every collective is an identity, so the shard IS the whole gradient (views,
        # no reduce-scatter / all-gather / copies)
        self._solo = info.world_size <= 1
        # reduce-scatter targets: the owned rows' summed gradients (fp32 for Adam)
        if self._solo:
            self.g_dec_shard = e.g_dec.view(G * n, d)
            self.g_enc_shard = e.g_enc.view(G * n, d) if kind == "untied" else None
        else:
            self.g_dec_shard = torch.empty(rows, d, device=dev)
            self.g_enc_shard = torch.empty(rows, d, device=dev) if kind == "untied" else None
        self._lowp = grad_dtype != torch.float32 and not self._solo
        if self._lowp:  # bf16 transport (all-to-all), fp32 accumulation on the row owner
            self._rs_in = [torch.empty(G * n * d, device=dev, dtype=grad_dtype) for _ in range(2 if kind == "untied" else 1)]
            self._rs_out = [torch.empty(info.world_size * rows * d, device=dev, dtype=grad_dtype) for _ in self._rs_in]
        self.graph = graph
        self.x_static = x_static
        self._graphs = {}
        self._ag = _Pending()  # shadow all-gathers of the last update (waited before the next compute)
        self.steps = 0

    # ------------------------------------------------------------------ ChunkedDataParallel hooks
    def set_grad_scale(self, s: float):
        self.engine.grad_scale = s

    def params(self):
        return list(self.engine.params.values())

    def after_param_sync(self):
        self.engine.refresh_shadows()

    def _region(self, key, fn):
        graphed_region(self, key, fn)

    def compute_grads(self, x):
        e = self.engine
        self._ag.wait()  # the previous update's shadows must have arrived
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
            e.wgrad_second(xp, reduce_bias=True)

        self._region("grads", run)
        return e.grad_all

    def reduce_async(self):
        """Reduce-scatter the weight gradients onto the row owners, all-reduce the bias (and
        loss-side extras); returns a _Pending whose completion means the shards are ready."""
        e = self.engine
        pend = _Pending()
        if self._solo:
            return pend
        G, n, d = e.n_models, e.n, e.d
        srcs = [e.g_dec] + ([e.g_enc] if e.kind == "untied" else [])
        dsts = [self.g_dec_shard] + ([self.g_enc_shard] if e.kind == "untied" else [])
        for i, (src, dst) in enumerate(zip(srcs, dsts)):
            if self._lowp:
                pend.add(*reduce_scatter_lowp(dst, src, self._rs_in[i], self._rs_out[i]))
            else:
                pend.add(reduce_scatter_async(dst.view(-1), src.reshape(-1)))
        # untied: _g_flat = [g_enc | g_bias]; tied: [g_dict | g_bias | extras] -- the tail is small
        pend.add(dist.all_reduce(e._g_flat[G * n * d:], async_op=True))
        return pend

    def apply_update(self, _payload=None):
        e = self.engine

        def run():
            self._shard_adam()
            e._bias_loss(update=True, reduced=True)

        self._region("update", run)
        e._host_step()
        self._issue_gathers()
        self.steps += 1
        return e.out

    # ------------------------------------------------------------------ internals
    def _shard_adam(self):
        from ..ops import adam as adam_ops

        e = self.engine
        G, n, d = e.n_models, e.n, e.d
        lo, hi = self.lo, self.hi
        rows = lambda t: t.view(G * n, d)[lo:hi]  # noqa: E731
        if e.kind == "untied":
            sets = [dict(p=rows(e.params["decoder"]), g=self.g_dec_shard, m=rows(e.m["decoder"]),
                         v=rows(e.v["decoder"]), shadow=rows(e.dec_shadow), norms=e.norms.view(-1)[lo:hi], norm=True),
                    dict(p=rows(e.params["encoder"]), g=self.g_enc_shard, m=rows(e.m["encoder"]),
                         v=rows(e.v["encoder"]), shadow=rows(e.enc_shadow), norms=None, norm=False)]
        else:
            sets = [dict(p=rows(e.params["encoder"]), g=self.g_dec_shard, m=rows(e.m["encoder"]),
                         v=rows(e.v["encoder"]), shadow=rows(e.enc_shadow), norms=e.norms.view(-1)[lo:hi], norm=True)]
        adam_ops.adam_rows(sets, e.lr, e.step_count + 1, *e.betas, e.eps, rows_per_model=n, step_dev=e.step_dev,
                           row0=lo, live=e.nactive)

    def _issue_gathers(self):
        if self._solo:
            return
        e = self.engine
        G, n, d = e.n_models, e.n, e.d
        lo, hi = self.lo, self.hi
        shadows = [e.dec_shadow] if e.kind == "untied" else []
        shadows.append(e.enc_shadow)
        for sh in shadows:
            self._ag.add(all_gather_async(sh.view(-1), lo * d, hi * d))
        # norms travel too (cheap) so every rank's copy is valid for exports / refreshes
        self._ag.add(all_gather_async(e.norms.view(-1), lo, hi))

    def gather_masters(self):
        """All-gather the fp32 masters and moments (exports / checkpoints): afterwards every
        rank holds the complete, current optimizer state."""
        self._ag.wait()
        if self._solo:
            return
        e = self.engine
        G, n, d = e.n_models, e.n, e.d
        lo, hi = self.lo, self.hi
        keys = ["decoder", "encoder"] if e.kind == "untied" else ["encoder"]
        for store in (e.params, e.m, e.v):
            for k in keys:
                w = all_gather_async(store[k].view(-1), lo * d, hi * d)
                if w is not None:
                    w.wait()


class ZeroEagerChunk:
    """ZeRO-1 over a flat parameter vector for an eager ``FunctionalEnsemble`` (any signature):
    rank r keeps Adam moments only for its 1/N slice of the flattened (padded) parameters, and
    all-gathers the updated parameters.  Elementwise Adam (torchopt semantics, the ensemble's
    own lr / betas / eps), so it equals the single-process optimizer on the global batch."""

    def __init__(self, ensemble, info: DistInfo, grad_dtype: torch.dtype = torch.float32):
        self.ens = ensemble
        self.info = info
        self.grad_dtype = grad_dtype
        self.scale = 1.0
        self.last = None
        leaves, self._spec = pytree.tree_flatten(ensemble.params)
        self._shapes = [t.shape for t in leaves]
        self._numel = sum(t.numel() for t in leaves)
        N = max(1, info.world_size)
        self._padded = -(-self._numel // N) * N
        self.lo, self.hi = shard_range(self._padded, info.rank, N)
        dev = leaves[0].device
        self.flat = torch.zeros(self._padded, device=dev)
        kw = ensemble.optimizer_kwargs
        self.lr = float(kw.get("lr", 1e-3))
        self.b1, self.b2 = kw.get("betas", (0.9, 0.999))
        self.eps = float(kw.get("eps", 1e-8))
        self.eps_root = float(kw.get("eps_root", 0.0))
        self.m = torch.zeros(self.hi - self.lo, device=dev)
        self.v = torch.zeros_like(self.m)
        self.count = 0
        self._gshard = torch.empty_like(self.m)
        self._pad_grad = torch.zeros(self._padded, device=dev)
        if grad_dtype != torch.float32:  # bf16 transport, fp32 owner accumulation
            self._send = torch.empty(self._padded, device=dev, dtype=grad_dtype)
            self._recv = torch.empty(self._padded, device=dev, dtype=grad_dtype)

    def set_grad_scale(self, s: float):
        self.scale = s

    def state_dict(self):
        """The full (unsharded) Adam state: every rank's moment slices all-gathered into padded
        flat vectors (collective: every rank calls it), so a checkpoint restores at any world size."""
        full = {}
        for k, t in (("m", self.m), ("v", self.v)):
            flat = torch.zeros(self._padded, device=t.device)
            flat[self.lo:self.hi] = t
            if dist.is_initialized() and self.info.world_size > 1:
                w = all_gather_async(flat, self.lo, self.hi)
                if w is not None:
                    w.wait()
            full[k] = flat[: self._numel].clone()
        full["count"] = self.count
        return full

    def load_state_dict(self, st):
        """Restore this rank's slices from a ``state_dict()`` (written at any world size)."""
        for k, t in (("m", self.m), ("v", self.v)):
            flat = torch.zeros(self._padded, device=t.device)
            flat[: self._numel] = st[k].to(t.device)
            t.copy_(flat[self.lo:self.hi])
        self.count = int(st["count"])

    def params(self):
        return [t.data for t in pytree.tree_leaves(self.ens.params)]

    def after_param_sync(self):
        pass

    def compute_grads(self, x):
        grads, (loss, aux) = self.ens.compute_grads(x)
        self.last = loss
        g = torch.cat([t.reshape(-1) for t in pytree.tree_leaves(grads)])
        self._pad_grad[: self._numel].copy_(g * self.scale)
        return self._pad_grad

    def reduce_async(self):
        pend = _Pending()
        if dist.is_initialized() and self.grad_dtype != torch.float32:
            pend.add(*reduce_scatter_lowp(self._gshard, self._pad_grad, self._send, self._recv))
        elif dist.is_initialized():  # (gloo with CUDA tensors: through an all-reduce)
            pend.add(reduce_scatter_async(self._gshard, self._pad_grad))
        else:
            self._gshard.copy_(self._pad_grad[self.lo:self.hi])
        return pend

    def apply_update(self, _payload=None):
        self.count += 1
        g = self._gshard
        b1, b2 = self.b1, self.b2
        self.m.mul_(b1).add_(g, alpha=1 - b1)
        self.v.mul_(b2).addcmul_(g, g, value=1 - b2)
        bc1, bc2 = 1 - b1 ** self.count, 1 - b2 ** self.count
        leaves = pytree.tree_leaves(self.ens.params)
        self.flat[: self._numel].copy_(torch.cat([t.reshape(-1) for t in leaves]))
        shard = self.flat[self.lo:self.hi]
        shard.add_(-self.lr * (self.m / bc1) / (torch.sqrt(self.v / bc2 + self.eps_root) + self.eps))
        if dist.is_initialized():
            w = all_gather_async(self.flat, self.lo, self.hi)
            if w is not None:
                w.wait()
        off = 0
        for t in leaves:
            k = t.numel()
            t.data.copy_(self.flat[off:off + k].view_as(t))
            off += k
        return self.last
