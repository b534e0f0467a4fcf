"""``UnrolledEnsemble``: LISTA and residual-denoising SAEs for a whole
ensemble on the grouped MFMA GEMM.

Reference: ``autoencoders/residual_denoising_autoencoder.py:9-122`` (LISTA layers with
shrinkage and momentum, https://arxiv.org/pdf/2008.02683.pdf) and ``:125-201`` (residual
denoising layers), trained by ``FunctionalEnsemble`` = ``vmap(grad(loss))`` per model.

Here every model's parameters are stacked on a leading model axis and the loss of all models
is written once in batched form.  Each layer's matrix products are grouped GEMMs over the
model axis (``grouped_mm``: one ``csrc/sae_gemm`` launch per product -- bf16 MFMA operands,
fp32 accumulation -- forward and both backward products); each LISTA layer's shrinkage +
momentum is one fused HIP pass forward and one backward (``lista_step``); the residual layers'
ReLU and the losses stay in torch autograd.  Adam is the reference's (torchopt)
update applied to the stacked tensors with a per-model learning rate.  Off the GPU, or when a
shape is not tiled by the kernels (B, n, d multiples of 128), the products fall back to fp32
``torch.matmul`` -- the CPU tests pin the engine against ``FunctionalEnsemble`` that way.
"""

from __future__ import annotations

from typing import Dict, List

import torch
import torch.nn.functional as F

from ..models.lista import (FunctionalLISTADenoisingSAE, FunctionalResidualDenoisingSAE, shrinkage)
from ..models.signatures import unit_rows


def _hip_ok(*dims) -> bool:
    return all(int(x) % 128 == 0 for x in dims)


# bf16 copies of the step's weight operands (D and the layer matrices feed several products
# forward and backward): one cast per tensor per step instead of one per product.  Keyed on
# storage pointer, shape and autograd version, and active only inside ``UnrolledEnsemble.grads``
# (every weight operand stays alive until its backward is done; the cache is cleared after).
_BF16_CACHE: dict = {}
_CACHE_ON = [False]


def _bf16_operand(t: torch.Tensor, cache: bool) -> torch.Tensor:
    if t.dtype == torch.bfloat16:
        return t.contiguous()
    if not (cache and _CACHE_ON[0]):
        return t.to(torch.bfloat16).contiguous()
    key = (t.data_ptr(), tuple(t.shape), t.stride(), t._version)
    hit = _BF16_CACHE.get(key)
    if hit is None:
        hit = _BF16_CACHE[key] = t.to(torch.bfloat16).contiguous()
    return hit


def _gemm(a, b, tb: bool):
    """fp32 [G, M, N] = a @ (b^T if tb else b) with bf16 operands on the MFMA kernel.
    a: [G, M, K] (or [M, K] shared by every model); b: [G, N, K] if tb else [G, K, N]."""
    from ..ops import gemm as gemm_ops

    G = b.shape[0]
    M = a.shape[-2]
    N = b.shape[1] if tb else b.shape[2]
    out = torch.empty(G, M, N, device=b.device, dtype=torch.float32)
    ab = _bf16_operand(a, cache=False)
    bb = _bf16_operand(b, cache=True)  # b is always a weight operand (D or a layer matrix)
    if tb:
        gemm_ops.matmul_nt(ab, bb, out)
    else:
        if ab.dim() == 2:
            ab = ab.expand(G, *ab.shape).contiguous()
        gemm_ops.matmul_nn(ab, bb, out)
    return out


def _gemm_tn(a, b):
    """fp32 [G, K, N] = a^T @ b, a: [G, M, K], b: [G, M, N] (either may be [M, .] shared)."""
    from ..ops import gemm as gemm_ops

    G = a.shape[0] if a.dim() == 3 else b.shape[0]
    M, K, N = a.shape[-2], a.shape[-1], b.shape[-1]
    ab, bb = a.to(torch.bfloat16), b.to(torch.bfloat16)
    ab = ab.expand(G, M, K) if ab.dim() == 2 else ab
    bb = bb.expand(G, M, N) if bb.dim() == 2 else bb
    out = torch.empty(G, K, N, device=a.device, dtype=torch.float32)
    gemm_ops.matmul_tn(ab.contiguous(), bb.contiguous(), out)
    return out


class _GroupedMM(torch.autograd.Function):
    """out = a @ (b^T if tb else b) over the model axis, backward on the same kernels:
    tb:  da = g @ b (NN),   db = g^T a (TN);   not tb:  da = g @ b^T (NT),  db = a^T g (TN)."""

    @staticmethod
    def forward(ctx, a, b, tb):
        ctx.tb = tb
        ctx.save_for_backward(a, b)
        return _gemm(a, b, tb)

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        tb = ctx.tb
        da = db = None
        if ctx.needs_input_grad[0]:
            da = _gemm(g, b, tb=not tb)
            if a.dim() == 2:
                da = da.sum(0)
        if ctx.needs_input_grad[1]:
            db = _gemm_tn(g, a) if tb else _gemm_tn(a, g)
        return da, db, None


def grouped_mm(a: torch.Tensor, b: torch.Tensor, tb: bool = False) -> torch.Tensor:
    """Batched a @ b (``tb``: a @ b^T) with autograd; the MFMA kernel when on the GPU and tiled."""
    M, K = a.shape[-2], a.shape[-1]
    N = b.shape[1] if tb else b.shape[2]
    if b.is_cuda and _hip_ok(M, N, K):
        return _GroupedMM.apply(a, b, tb)
    return torch.matmul(a, b.transpose(-1, -2) if tb else b)


class _ListaStep(torch.autograd.Function):
    """One LISTA layer's elementwise part in one HIP pass each way (csrc/elementwise.hip):
    r = y + a, x_ = shrink(r, theta), y' = x_ + m (x_ - xs); returns (y', x_)."""

    @staticmethod
    def forward(ctx, y, a, xs, theta, m):
        from ..ops import _lib

        ctx.set_materialize_grads(False)
        y, a, xs, theta, m = (t.contiguous() for t in (y, a, xs, theta, m))
        G, B, n = y.shape
        xo, yo = torch.empty_like(y), torch.empty_like(y)
        p = _lib.ptr
        _lib.check(_lib.lib().sc_lista_fwd(p(y), p(a), p(xs), p(theta), p(m), p(xo), p(yo), G, B, n,
                                           _lib.stream_handle()), "sc_lista_fwd")
        ctx.save_for_backward(y, a, xs, theta, m)
        return yo, xo

    @staticmethod
    def backward(ctx, gy, gx):
        from ..ops import _lib

        y, a, xs, theta, m = ctx.saved_tensors
        G, B, n = y.shape
        if gy is None:
            gy = torch.zeros_like(y)
        rb = 64 if B % 64 == 0 else 4
        gr, gxs = torch.empty_like(y), torch.empty_like(y)
        gth = torch.empty(G, B // rb, n, device=y.device)
        gm = torch.empty(G, B // rb, n // 256, device=y.device)
        p = _lib.ptr
        _lib.check(_lib.lib().sc_lista_bwd(p(gy.contiguous()), p(gx.contiguous() if gx is not None else None), p(y),
                                           p(a), p(xs), p(theta), p(m), p(gr), p(gxs), p(gth), p(gm), G, B, n, rb,
                                           _lib.stream_handle()), "sc_lista_bwd")
        return gr, gr, gxs, gth.sum(1), gm.sum((1, 2))


def lista_step(y, a, xs, theta, m):
    """(y', x_) of a LISTA layer for stacked [G, B, n] tensors (theta [G, n], m [G] clamped)."""
    G, B, n = y.shape
    if y.is_cuda and n % 256 == 0 and B % 4 == 0:
        return _ListaStep.apply(y, a, xs, theta, m)
    x_ = shrinkage(y + a, theta.unsqueeze(1))
    return x_ + m.view(-1, 1, 1) * (x_ - xs), x_


_KINDS = {FunctionalLISTADenoisingSAE: "lista", FunctionalResidualDenoisingSAE: "residual"}


def supports(sig) -> bool:
    return sig in _KINDS


class UnrolledEnsemble:
    def __init__(self, models, sig, lr=1e-3, device="cuda", betas=(0.9, 0.999), eps=1e-8):
        if sig not in _KINDS:
            raise ValueError(f"{sig} is not an unrolled-encoder signature")
        self.sig, self.kind = sig, _KINDS[sig]
        self.device = torch.device(device)
        self.n_models = G = len(models)
        dev = self.device
        p0 = models[0][0]
        self.n_layers = len(p0["encoder_layers"])
        st = lambda get: torch.stack([get(m[0]).detach().float() for m in models]).to(dev).contiguous()
        self.params: Dict[str, torch.Tensor] = {"decoder": st(lambda p: p["decoder"])}
        for i in range(self.n_layers):
            for k in p0["encoder_layers"][i]:
                self.params[f"layer{i}.{k}"] = st(lambda p, i=i, k=k: p["encoder_layers"][i][k])
        if self.kind == "residual":
            self.params["encoder_bias"] = st(lambda p: p["encoder_bias"])
        for t in self.params.values():
            t.requires_grad_(True)
        self.buffers = [dict(b) for _, b in models]
        self.l1 = torch.tensor([float(b["l1_alpha"]) for _, b in models], device=dev)
        lrs = lr if isinstance(lr, (list, tuple)) else [lr] * G
        self.lr = torch.tensor([float(x) for x in lrs], device=dev)
        self.betas, self.eps = betas, eps
        self.m = {k: torch.zeros_like(v) for k, v in self.params.items()}
        self.v = {k: torch.zeros_like(v) for k, v in self.params.items()}
        self.step_count = 0

    # ------------------------------------------------------------------ model
    def _layer(self, i, k):
        return self.params[f"layer{i}.{k}"]

    def encode_stacked(self, x: torch.Tensor) -> torch.Tensor:
        """Codes of every model [G, B, n] for a shared batch x [B, d] (autograd-tracked)."""
        D = unit_rows(self.params["decoder"])
        y = grouped_mm(x, D, tb=True)  # [G, B, n]
        if self.kind == "lista":
            xs = y
            for i in range(self.n_layers):
                m = torch.clamp(self._layer(i, "rho"), 0.0, 1.0)
                a = grouped_mm(x - grouped_mm(y, D), self._layer(i, "W"), tb=True)
                y, xs = lista_step(y, a, xs, self._layer(i, "theta"), m)
            return y
        c = y
        for i in range(self.n_layers):
            c = grouped_mm(F.relu(c + self._layer(i, "theta").unsqueeze(1)), self._layer(i, "W"), tb=True) + c
        return F.relu(c + self.params["encoder_bias"].unsqueeze(1))

    def losses(self, x: torch.Tensor):
        """Per-model (total, l_rec, l_l1) [G] and the codes -- the reference loss per model."""
        D = unit_rows(self.params["decoder"])
        c = self.encode_stacked(x)
        l_rec = (grouped_mm(c, D) - x).pow(2).mean(dim=(1, 2))
        l_l1 = self.l1 * c.abs().sum(-1).mean(-1)
        return l_rec + l_l1, l_rec, l_l1, c

    # ------------------------------------------------------------------ training
    def grads(self, x: torch.Tensor):
        """Gradients of every model's loss (models are independent: d(sum)/dθ_g = dL_g/dθ_g)."""
        x = x.to(self.device, torch.float32)
        _BF16_CACHE.clear()
        _CACHE_ON[0] = True
        try:
            total, l_rec, l_l1, c = self.losses(x)
            keys = list(self.params)
            gs = torch.autograd.grad(total.sum(), [self.params[k] for k in keys])
        finally:
            _CACHE_ON[0] = False
            _BF16_CACHE.clear()
        return dict(zip(keys, gs)), (total.detach(), l_rec.detach(), l_l1.detach(), c.detach())

    @torch.no_grad()
    def apply_grads(self, grads):
        """torchopt Adam (eps_root = 0) with a per-model learning rate."""
        self.step_count += 1
        b1, b2 = self.betas
        bc1 = 1.0 - b1 ** self.step_count
        bc2 = 1.0 - b2 ** self.step_count
        for k, p in self.params.items():
            g = grads[k]
            m, v = self.m[k], self.v[k]
            if p.is_cuda and p.dim() == 3 and p.shape[-1] % 256 == 0 and p.shape[-1] <= 4096:
                # matrices: the row-Adam kernel (one HBM pass; the torch form below is ~10)
                from ..ops import adam as adam_ops

                adam_ops.adam_rows([dict(p=p.data, g=g.contiguous(), m=m, v=v, shadow=None, norms=None, norm=False)],
                                   self.lr, self.step_count, b1, b2, self.eps)
                continue
            m.mul_(b1).add_(g, alpha=1.0 - b1)
            v.mul_(b2).addcmul_(g, g, value=1.0 - b2)
            lr = self.lr.view(-1, *([1] * (p.dim() - 1)))
            p.sub_(lr * (m / bc1) / ((v / bc2).sqrt() + self.eps))

    def step_batch(self, batch: torch.Tensor, expand_dims: bool = True):
        grads, (total, l_rec, l_l1, c) = self.grads(batch)
        self.apply_grads(grads)
        return {"loss": total, "l_reconstruction": l_rec, "l_l1": l_l1}, {"c": c}

    # ------------------------------------------------------------------ export / state
    def unstack(self, device="cpu") -> List[tuple]:
        out = []
        for g in range(self.n_models):
            get = lambda k: self.params[k][g].detach().to(device).clone()
            p = {"decoder": get("decoder"),
                 "encoder_layers": [{k.split(".", 1)[1]: get(k) for k in self.params if k.startswith(f"layer{i}.")}
                                    for i in range(self.n_layers)]}
            if self.kind == "residual":
                p["encoder_bias"] = get("encoder_bias")
            b = {k: (v.detach().to(device).clone() if torch.is_tensor(v) else v) for k, v in self.buffers[g].items()}
            out.append((p, b))
        return out

    def to_learned_dicts(self, device="cpu"):
        return [self.sig.to_learned_dict(p, b) for p, b in self.unstack(device)]

    def state_dict(self):
        return {"params": {k: v.detach() for k, v in self.params.items()}, "m": self.m, "v": self.v,
                "step": self.step_count}

    def load_state_dict(self, sd):
        with torch.no_grad():
            for name in ("params", "m", "v"):
                for k, t in sd[name].items():
                    getattr(self, name)[k].copy_(t)
        self.step_count = int(sd["step"])
