"""``EnsembleTrainer``: one facade over the three training engines.

* ``FusedSAEEnsemble`` (gfx950 kernels) for untied / tied / masked SAEs and the SAE
  step of ``FunctionalFista``;
* ``FusedTopKEnsemble`` (gfx950 kernels) for ``TopKEncoder`` with per-model k;
* ``UnrolledEnsemble`` (grouped MFMA GEMMs + torch autograd) for LISTA / residual-denoising SAEs;
* ``FunctionalEnsemble`` (eager torch.func, CPU or GPU) for everything else and as
  the CPU oracle.

``engine="auto"`` picks the fused path on a GPU when the shapes fit the kernels
(B % 128, n % 128, d % 256) and otherwise falls back to eager -- explicitly, with
the reason recorded in ``trainer.engine_reason``.  The FISTA dictionary update of
the fork (reference ``big_sweep.py:176-198``) is a post-step hook.
"""

from __future__ import annotations

from typing import Any, Dict, List, Optional, Sequence, Tuple

import torch

from ..models.fista import FistaDictUpdater, FunctionalFista
from ..models.signatures import unit_rows
from ..models.topk import TopKEncoder
from . import analytic, unrolled
from .ensemble import FunctionalEnsemble
from .optim import adam


def _fused_ok(models, sig, batch_size, device) -> Tuple[bool, str]:
    if not (torch.cuda.is_available() and torch.device(device).type == "cuda"):
        return False, "no GPU"
    from ..ops import _lib

    if not _lib.available():
        raise RuntimeError("GPU present but the gfx950 kernel library failed to load")
    p0, b0 = models[0]
    key = "dict" if sig is TopKEncoder else "encoder"
    if key not in p0:
        return False, f"signature {sig.__name__} has no '{key}' parameter"
    n, d = p0[key].shape
    if batch_size % 128 or n % 128 or d % 256:
        return False, f"shape B={batch_size}, n={n}, d={d} not tiled by the fused kernels"
    if sig is TopKEncoder:
        return True, "fused top-k"
    if getattr(sig, "fused_kind", None) is None:
        return False, f"no fused kernels for {sig.__name__}"
    return True, f"fused {sig.fused_kind} SAE"


class EnsembleTrainer:
    def __init__(self, models: List[Tuple[dict, dict]], sig, lr: float = 1e-3, batch_size: int = 256,
                 device="cuda", engine: str = "auto", name: str = "ensemble", args: Optional[dict] = None,
                 fista_iters: int = 500, fista_backend: str = "auto", persist_hessian: bool = False,
                 basis_normalize: str = "column", use_graph: bool = False, fista_eta: str = "tracked",
                 dist=None, parallel: str = "none", objective: str = "loss", fista_loss_iters: int = 50):
        """``objective="fista_loss"`` (FunctionalFista only): the "FISTA in the loss" variant
        (reference autoencoders/fista.py:141-172) on ``FistaLossEnsemble`` -- tied normalised
        SAE loss plus the residual of ``fista_loss_iters`` unrolled FISTA iterations."""
        self.sig = sig
        self.name = name
        self.args = dict(args or {})
        self.batch_size = batch_size
        self.device = torch.device(device)
        self.n_models = len(models)
        self.meta = [dict(b) for _, b in models]
        self.es = None
        self.dp = None
        self.local = slice(0, len(models))
        if parallel in ("dp", "zero1"):
            # data parallel over the ranks (each rank passes its own rows to `step`): on MI355X the
            # fused engine with the RCCL collectives captured in its step graph (parallel/graphed.py,
            # native communicator); elsewhere the eager ensemble with gloo / ProcessGroup collectives
            if objective != "loss" or sig is FunctionalFista:
                raise ValueError("parallel='dp'/'zero1' trains the SAE objectives (no FISTA hooks)")
            self._init_dp(models, sig, lr, batch_size, device, engine, dist, parallel)
        elif parallel == "es":
            # ensemble-axis sharding (parallel/ensemble_shard.py): this rank trains its block
            # of the models on the all-gathered global batch; `step` takes this rank's rows
            self._init_sharded(models, sig, lr, batch_size, device, engine, dist, use_graph)
            models = list(models[self.local])
        elif parallel != "none":
            raise ValueError(f"parallel must be 'none', 'es', 'dp' or 'zero1', got {parallel!r}")
        if objective not in ("loss", "fista_loss"):
            raise ValueError(f"objective must be 'loss' or 'fista_loss', got {objective!r}")
        if objective == "fista_loss" and (sig is not FunctionalFista or parallel != "none"):
            raise ValueError("objective='fista_loss' needs the FunctionalFista signature and parallel='none'")
        if objective == "fista_loss":
            ok, why = False, "fista-in-loss engine"  # its own engines below (fused or autograd)
        else:
            ok, why = _fused_ok(models, sig, batch_size, device) if engine in ("auto", "fused") else (False, "eager")
        if engine == "fused" and not ok and objective != "fista_loss":
            raise ValueError(f"fused engine requested but unavailable: {why}")
        self.engine_reason = why
        self.kind = "eager"
        if self.dp is not None:
            self.kind = self._dp_kind
        elif self.es is not None:
            self.impl = self.es.engine
            self.kind = self._es_kind
        elif objective == "fista_loss":
            from .fista_loss import FistaLossEnsemble, FusedFistaLossEnsemble, fused_ok

            fok = fista_backend != "torch" and fused_ok(models, batch_size, device, fista_loss_iters)
            if engine == "fused" and not fok:
                raise ValueError("fused FISTA-in-loss engine requested but unavailable (needs the GPU kernels, "
                                 "B % 128 == 0, d % 256 == 0, n <= d and n in the Gram kernel's sizes)")
            if engine in ("auto", "fused") and fok:
                self.impl = FusedFistaLossEnsemble(models, lr=lr, batch_size=batch_size, device=device,
                                                   num_iter=fista_loss_iters)
                self.kind = "fista-loss-fused"
                self.engine_reason = "fused fista-in-loss"
            else:
                self.impl = FistaLossEnsemble(models, lr=lr, batch_size=batch_size, device=device,
                                              num_iter=fista_loss_iters, backend=fista_backend)
                self.kind = "fista-loss"
        elif ok and sig is TopKEncoder:
            from .topk import FusedTopKEnsemble

            self.impl = FusedTopKEnsemble(models, sig, lr=lr, batch_size=batch_size, device=device)
            self.kind = "fused-topk"
        elif ok:
            from .fused import FusedSAEEnsemble

            self.impl = FusedSAEEnsemble(models, sig, lr=lr, batch_size=batch_size, device=device)
            if use_graph:
                self.impl.enable_graph()
            self.kind = "fused-sae"
        elif engine in ("auto", "unrolled") and unrolled.supports(sig):
            # LISTA / residual-denoising SAEs: the stacked batched loss on the grouped MFMA GEMM
            self.impl = unrolled.UnrolledEnsemble(models, sig, lr=lr, device=device)
            self.kind = "unrolled"
        elif engine in ("auto", "analytic") and analytic.supports(sig):
            # closed-form gradients with batched GEMMs (no vmap/autograd): the CPU fast path
            self.impl = analytic.AnalyticSAEEnsemble(models, sig, lr=lr, device=device)
            self.kind = "analytic"
        else:
            self.impl = FunctionalEnsemble(models, sig, adam, {"lr": lr}, device=device,
                                           no_stacking=sig is TopKEncoder)
        self.fista = None
        if sig is FunctionalFista and objective == "loss":
            self.fista = FistaDictUpdater(num_iter=fista_iters, persist_hessian=persist_hessian,
                                          normalize=basis_normalize, backend=fista_backend, eta_method=fista_eta)
        self.last_loss = None
        self.last_losses: Dict[str, torch.Tensor] = {}
        self.steps = 0

    def _init_dp(self, models, sig, lr, batch_size, device, engine, dist, mode):
        from ..parallel.dist import DistInfo

        info = dist if dist is not None else DistInfo(device=torch.device(device))
        fused, _ = _fused_ok(models, sig, batch_size, device) if engine in ("auto", "fused") else (False, "")
        if fused and sig is not TopKEncoder and getattr(sig, "fused_kind", None) in ("untied", "tied"):
            from ..parallel.graphed import GraphedDataParallel
            from ..parallel.rccl import RcclComm
            from .fused import FusedSAEEnsemble

            # flat fp32 gradients: the reductions read grad_all (no split-K slabs for this shape)
            eng = FusedSAEEnsemble(models, sig, lr=lr, batch_size=batch_size, device=device, wgrad_split=1)
            if info.world_size > 1 and info.backend == "gloo":
                from ..parallel.host_comm import HostComm

                self._comm = HostComm(info)  # gloo ranks (e.g. sharing one GPU): host-staged, eager steps
            else:
                self._comm = RcclComm(info)
            self.dp = GraphedDataParallel([eng], info, self._comm, None, mode=mode)
            self.impl = eng
            self._dp_kind = f"{mode}-graphed"
            return
        from ..parallel.data_parallel import ChunkedDataParallel, DataParallelEnsemble, EagerChunk
        from ..parallel.zero import ZeroEagerChunk

        ens = FunctionalEnsemble(models, sig, adam, {"lr": lr}, device=device)
        self.impl = ens
        if mode == "zero1":
            self.dp = ChunkedDataParallel([ZeroEagerChunk(ens, info)], info)
        else:
            self.dp = DataParallelEnsemble(ens, info)
        self._dp_kind = f"{mode}-eager"

    def _init_sharded(self, models, sig, lr, batch_size, device, engine, dist, use_graph):
        from ..parallel.dist import DistInfo
        from ..parallel.ensemble_shard import EnsembleSharded, shard_range

        info = dist if dist is not None else DistInfo(device=torch.device(device))
        lo, hi = shard_range(len(models), info)
        self.local = slice(lo, hi)
        d = models[0][0]["encoder"].shape[1]
        gb = batch_size * info.world_size
        fused, _ = _fused_ok(list(models[lo:hi]), sig, gb, device) if engine in ("auto", "fused") else (False, "")
        if fused and sig is not TopKEncoder:
            from .fused import FusedSAEEnsemble

            def factory(ms, bs):
                return FusedSAEEnsemble(ms, sig, lr=lr, batch_size=bs, device=device)
            self._es_kind = "fused-sae"
            dtype = torch.bfloat16
        elif analytic.supports(sig):
            def factory(ms, bs):
                return analytic.AnalyticSAEEnsemble(ms, sig, lr=lr, device=device)
            self._es_kind = "analytic"
            dtype = torch.float32
        else:
            raise ValueError(f"ensemble sharding supports the SAE signatures, not {sig.__name__}")
        self.es = EnsembleSharded(models, factory, info, batch_per_rank=batch_size, d=d, dtype=dtype)
        if use_graph and self._es_kind == "fused-sae":
            self.es.enable_graph()

    # ------------------------------------------------------------------ training
    def step(self, batch: torch.Tensor) -> torch.Tensor:
        """One optimizer step of every model; returns per-model total loss [G] on device
        (with ensemble sharding: of this rank's models, on the gathered global batch)."""
        if self.dp is not None:  # data parallel: `batch` is this rank's rows
            if self.kind.endswith("graphed"):
                out = self.dp.step_batch(batch)[0]
                self.last_losses = {"loss": out[:, 0], "l_reconstruction": out[:, 1], "l_l1": out[:, 2],
                                    "l_bias_decay": out[:, 3], "l0": out[:, 4]}
            else:
                res = self.dp.step_batch(batch.to(self.device, torch.float32))
                loss = res[0]  # (loss, aux) of the eager DP wrapper / the chunk losses of ZeRO-1
                self.last_losses = dict(loss) if isinstance(loss, dict) else {"loss": loss}
            self.steps += 1
            self.last_loss = self.last_losses["loss"]
            return self.last_loss
        if self.es is not None:
            x = batch.to(self.device, self.es.gbuf[0].dtype)
            out = self.es.step_batch(x)
            if self.kind == "fused-sae":
                self.last_losses = {"loss": out[:, 0], "l_reconstruction": out[:, 1], "l_l1": out[:, 2],
                                    "l_bias_decay": out[:, 3], "l0": out[:, 4]}
                codes = None
            else:
                loss, aux = out
                self.last_losses = dict(loss)
                codes = aux.get("c") if isinstance(aux, dict) else None
            if self.fista is not None:
                self._fista_update(self.es.gbuf[1 - self.es._cur], codes)  # the gathered batch just used
            self.steps += 1
            self.last_loss = self.last_losses["loss"]
            return self.last_loss
        if self.kind == "fused-sae":
            out = self.impl.step_batch(batch)
            self.last_losses = {"loss": out[:, 0], "l_reconstruction": out[:, 1], "l_l1": out[:, 2],
                                "l_bias_decay": out[:, 3], "l0": out[:, 4]}
            codes = None
        elif self.kind == "fused-topk":
            mse = self.impl.step_batch(batch)
            self.last_losses = {"loss": mse}
            codes = None
        elif self.kind in ("fista-loss", "fista-loss-fused"):
            total = self.impl.step_batch(batch)
            self.last_losses = {"loss": total, **self.impl.last}
            codes = None
        else:
            loss, aux = self.impl.step_batch(batch.to(self.device, torch.float32))
            self.last_losses = dict(loss)
            codes = aux.get("c") if isinstance(aux, dict) else None
        if self.fista is not None:
            self._fista_update(batch, codes)
        self.steps += 1
        self.last_loss = self.last_losses["loss"]
        return self.last_loss

    def _fista_update(self, batch, codes):
        if self.kind == "fused-sae":
            eng = self.impl
            # the bf16 batch as it is (the GPU FISTA path multiplies bf16 operands; no fp32 copy)
            x = batch.to(self.device) if batch.dtype == torch.bfloat16 else batch.to(self.device, torch.float32)
            new, _, _ = self.fista(eng.params["decoder"], x, eng.c, eng.l1)
            eng.params["decoder"].copy_(new)
            eng.refresh_decoder_shadow()
            return
        x = batch.to(self.device, torch.float32)
        ens = self.impl
        l1 = ens.buffers["l1_alpha"]
        new, _, _ = self.fista(ens.params["decoder"], x, codes.float(), l1)
        ens.params["decoder"].data.copy_(new)

    # ------------------------------------------------------------------ export / state
    def hyperparams(self, ensemble_hyperparams: Sequence[str] = (), buffer_hyperparams: Sequence[str] = ("l1_alpha",),
                    local: bool = False) -> List[dict]:
        """Per-model hyper-parameters (``local``: only this rank's models under ensemble sharding)."""
        out = []
        for meta in (self.meta[self.local] if local else self.meta):
            hp = {}
            for k in ensemble_hyperparams:
                if k not in self.args:
                    raise ValueError(f"Hyperparameter {k} not found in args")
                hp[k] = self.args[k]
            for k in buffer_hyperparams:
                if k in meta:
                    v = meta[k]
                    hp[k] = v.item() if torch.is_tensor(v) else v
            out.append(hp)
        return out

    def to_learned_dicts(self, ensemble_hyperparams=("dict_size",), buffer_hyperparams=("l1_alpha",),
                         device="cpu") -> List[Tuple[Any, dict]]:
        """Every model's LearnedDict (a collective under ensemble sharding: all ranks call it)."""
        if self.es is not None:
            lds = self.es.to_learned_dicts(self.meta, self.sig, device)
            return list(zip(lds, self.hyperparams(ensemble_hyperparams, buffer_hyperparams)))
        if self.dp is not None and self.kind.endswith("graphed"):
            lds = self.dp.to_learned_dicts(device)
            return list(zip(lds, self.hyperparams(ensemble_hyperparams, buffer_hyperparams)))
        lds = self.impl.to_learned_dicts(device)
        return list(zip(lds, self.hyperparams(ensemble_hyperparams, buffer_hyperparams)))

    def losses_host(self) -> List[Dict[str, float]]:
        """Per-model loss dicts of the last step.  Under ensemble sharding only this rank's
        models (``self.local``) have losses here, matching ``hyperparams(local=True)``."""
        host = {k: v.detach().float().cpu() for k, v in self.last_losses.items() if torch.is_tensor(v)}
        count = (self.local.stop - self.local.start) if self.es is not None else self.n_models
        return [{k: float(v[i]) for k, v in host.items()} for i in range(count)]

    def close(self):
        """Release the data-parallel communicator: synchronise, drop the captured graphs that hold its
        collectives, then destroy it (idempotent; the GC never has to)."""
        comm = getattr(self, "_comm", None)
        if comm is None:
            return
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        if self.dp is not None and hasattr(self.dp, "_graphs"):
            self.dp._graphs = {}
        comm.close()
        self._comm = None

    def state_dict(self) -> Dict[str, Any]:
        st = {"kind": self.kind, "steps": self.steps, "name": self.name, "args": self.args}
        if self.kind == "zero1-eager":
            # the sharded moments gathered whole (collective: every rank calls state_dict)
            from torch.utils import _pytree as pytree

            st["impl"] = {"params": pytree.tree_map(lambda t: t.detach().clone(), self.impl.params),
                          "zero": [c.state_dict() for c in self.dp.chunks]}
        elif self.kind.endswith("-graphed"):
            self.dp.gather_masters()  # ZeRO-1: every rank's masters / moments complete
            st["impl"] = self.impl.state_dict()
        elif self.kind == "fused-sae":
            st["impl"] = self.impl.state_dict()
        elif self.kind == "fused-topk":
            st["impl"] = {"params": self.impl.params, "m": self.impl.m, "v": self.impl.v,
                          "step": self.impl.step_count}
        elif self.kind in ("analytic", "fista-loss", "fista-loss-fused", "unrolled"):
            st["impl"] = self.impl.state_dict()
        else:
            st["impl"] = {"params": self.impl.params, "optim": self.impl.optim_states}
        if self.fista is not None and self.fista.hessian is not None:
            st["hessian"] = self.fista.hessian
        return st

    def load_state_dict(self, st: Dict[str, Any]):
        if st["kind"] != self.kind:
            raise ValueError(f"checkpoint engine {st['kind']} != {self.kind}")
        self.steps = int(st["steps"])
        imp = st["impl"]
        if self.kind in ("fused-sae", "analytic", "fista-loss", "fista-loss-fused", "unrolled", "dp-graphed",
                         "zero1-graphed"):
            self.impl.load_state_dict(imp)
        elif self.kind == "zero1-eager":
            from torch.utils import _pytree as pytree

            for a, b in zip(pytree.tree_leaves(self.impl.params), pytree.tree_leaves(imp["params"])):
                a.data.copy_(b)
            for c, zst in zip(self.dp.chunks, imp["zero"]):
                c.load_state_dict(zst)
        elif self.kind == "fused-topk":
            for d_ in ("params", "m", "v"):
                for k, t in imp[d_].items():
                    getattr(self.impl, d_)[k].copy_(t)
            self.impl.step_count = int(imp["step"])
            self.impl.step_dev.fill_(self.impl.step_count)
            from ..ops import adam as adam_ops

            adam_ops.shadow_rows(self.impl.params["dict"], self.impl.shadow, self.impl.norms, normalize=True)
        else:
            from torch.utils import _pytree as pytree

            for a, b in zip(pytree.tree_leaves(self.impl.params), pytree.tree_leaves(imp["params"])):
                a.data.copy_(b)
            for a, b in zip(pytree.tree_leaves(self.impl.optim_states), pytree.tree_leaves(imp["optim"])):
                a.copy_(b)
        if "hessian" in st and self.fista is not None:
            self.fista.hessian = st["hessian"].to(self.device)
