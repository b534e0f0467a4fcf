"""``UnrolledEnsemble``: LISTA and residual-denoising SAEs for a whole
ensemble on the grouped MFMA GEMM.

Reference: ``autoencoders/residual_denoising_autoencoder.py:9-122`` (LISTA layers with
shrinkage and momentum, https://arxiv.org/pdf/2008.02683.pdf) and ``:125-201`` (residual
denoising layers), trained by ``FunctionalEnsemble`` = ``vmap(grad(loss))`` per model.

On the GPU both families train through ``UnrolledEnsemble._fused_step``: the forward and a hand-derived
backward with no autograd, every product a grouped MFMA GEMM whose epilogue writes the operand the
next product reads (bf16 residuals, bf16 code gradients, alpha-scaled signs folded in), the
shrinkage/momentum of each layer one HIP pass each way (``sc_lista_fwd2`` / ``sc_lista_bwd2``: r, the
bf16 copy of y', the L1 sums, the summed incoming gradients, the first layer's y0 = xs0 gradient), and
the matrices' Adam the row kernel that also rewrites their bf16 shadows (the decoder's normalised:
the unit-row Jacobian is applied there); the residual family's ReLU layers likewise
(``sc_res_fwd`` / ``sc_res_bwd``).  The autograd path (``grads``) stays for the CPU, the tests and
shapes the kernels do not tile.

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


# the unrolled steps' weight gradients keep the automatic block shape (256x256 here: the eight-wave
# 256x128 layout default of the SAE step measured +1.4 % on LISTA, profiles/r6/wg14/)
_WG_CFG = 0


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
        # bf16 shadows of the matrices for the explicit LISTA step (built on first use, rewritten by
        # its Adam; dropped whenever the parameters change another way)
        self._mats = ["decoder"] + [f"layer{i}.W" for i in range(self.n_layers)]
        self._sh = None

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
        self._sh = None
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
        if self._fused_ok(batch.shape[0]):
            total, l_rec, l_l1, c = self._fused_step(batch)
        else:
            grads, (total, l_rec, l_l1, c) = self.grads(batch)
            self.apply_grads(grads)
        return {"loss": total, "l_reconstruction": l_rec, "l_l1": l_l1}, {"c": c}

    # ------------------------------------------------------------------ explicit LISTA step (GPU)
    def _fused_ok(self, B: int) -> bool:
        G, n, d = self.params["decoder"].shape
        return (self.device.type == "cuda" and B % 128 == 0 and n % 256 == 0 and d % 256 == 0 and d <= 4096
                and (B * n) % 1024 == 0 and (self.kind == "lista" or n <= 4096))

    def _shadows(self):
        from ..ops import adam as adam_ops

        if self._sh is None:
            self._sh = {}
            for k in self._mats:
                p = self.params[k].detach()
                self._sh[k] = torch.empty(p.shape, device=self.device, dtype=torch.bfloat16)
                adam_ops.shadow_rows(p, self._sh[k], normalize=(k == "decoder"))
        return self._sh

    @torch.no_grad()
    def _lista_fused_grads(self, x: torch.Tensor):
        """One LISTA training step of every model without autograd (see the module docstring).

        Forward, layer i (E = x - y D, y_0 = xs_0 = x D^T):  a = E W^T,  r = y + a,
        x_ = shrink(r, theta),  y' = x_ + m (x_ - xs);  c = y_L,  L = |c D - x|^2 / (B d) + l1 |c|_1 / B.
        Backward, layer i (incoming dy', dxs'):  dr = shrink'(r) ((1 + m) dy' + dxs'),
        dxs = -m dy',  dW = dr^T E,  dE = dr W,  dy = dr - dE D^T (+ dxs for i = 0),
        dD_hat += -y^T dE (+ dy_0^T x, + c^T dL/dx_hat);  theta / m from block partials.
        Reference: autoencoders/residual_denoising_autoencoder.py:26-36, :66-83."""
        from ..ops import _lib
        from ..ops import gemm as gemm_ops

        G, n, d = self.params["decoder"].shape
        B, L, dev = int(x.shape[0]), self.n_layers, self.device
        f32 = dict(device=dev, dtype=torch.float32)
        bf = dict(device=dev, dtype=torch.bfloat16)
        sh = self._shadows()
        Db = sh["decoder"]
        xb = x.to(dev, torch.bfloat16).contiguous()
        p = _lib.ptr
        st = _lib.stream_handle()
        rho = [self.params[f"layer{i}.rho"].detach() for i in range(L)]
        ms = [r.clamp(0.0, 1.0).contiguous() for r in rho]
        ths = [self.params[f"layer{i}.theta"].detach().contiguous() for i in range(L)]
        part = torch.empty(G, (B // 128) * (d // 128), **f32)
        absp = torch.empty(G * B * n // 1024, **f32)

        # ---- forward
        y = torch.empty(G, B, n, **f32)
        gemm_ops.matmul_nt(xb, Db, y)  # y_0 = x D^T
        yb, xs = y.to(torch.bfloat16), y
        saved = []
        for i in range(L):
            rneg = torch.empty(G, B, d, **bf)
            gemm_ops.decode_residual(yb, Db, xb, rneg, part)  # y D - x = -E
            a = torch.empty(G, B, n, **f32)
            gemm_ops.matmul_nt(rneg, sh[f"layer{i}.W"], a, alpha=-1.0)  # a = E W^T
            xo, yo, yob = torch.empty(G, B, n, **f32), torch.empty(G, B, n, **f32), torch.empty(G, B, n, **bf)
            _lib.check(_lib.lib().sc_lista_fwd2(p(y), p(a), p(xs), p(ths[i]), p(ms[i]), p(xo), p(yo), p(a), p(yob),
                                                p(absp) if i == L - 1 else None, G, B, n, st), "sc_lista_fwd2")
            saved.append((yb, a, xs, rneg))  # (a now holds r = y + a)
            y, yb, xs = yo, yob, xo
        c, cb = y, yb
        rf = torch.empty(G, B, d, **bf)
        gemm_ops.decode_residual(cb, Db, xb, rf, part)  # c D - x, with sum(r^2) partials
        l_rec = part.sum(1) / (B * d)
        l_l1 = self.l1 * absp.view(G, -1).sum(1) / B

        # ---- backward (the bf16 code gradients carry -dr, so every weight-gradient term has unit weight:
        # dW = (-dr)^T (-E), -dE = (-dr) W; the decoder's reconstruction term takes alpha r in bf16)
        alpha = 2.0 / (B * d)
        gc = torch.empty(G, B, n, **f32)
        gemm_ops.matmul_nt(rf, Db, gc, alpha=alpha)  # d l_rec / dc
        rb = 64
        gth_part = torch.empty(G, B // rb, n, **f32)
        gm_part = torch.empty(G, B // rb, n // 256, **f32)
        gth, grho = {}, {}
        dterms = [(cb, rf.mul(alpha))]  # decoder (D_hat) terms: c^T dL/dx_hat, then per layer
        wterms = {}
        gy, gy2, gx, l1c = gc, None, None, (self.l1 / B).float().contiguous()
        for i in reversed(range(L)):
            yb_i, r_i, xs_i, rneg_i = saved[i]
            first = i == 0
            ngrb = torch.empty(G, B, n, **bf)
            gr = None if first else torch.empty(G, B, n, **f32)
            gxs = None if first else torch.empty(G, B, n, **f32)
            ub = torch.empty(G, B, n, **bf) if first else None
            _lib.check(_lib.lib().sc_lista_bwd2(p(gy), p(gy2), p(gx), p(r_i), None, p(xs_i), p(ths[i]), p(ms[i]),
                                                p(l1c), p(gr), p(ngrb), -1.0, p(gxs), p(ub), p(gth_part), p(gm_part),
                                                G, B, n, rb, st), "sc_lista_bwd2")
            gth[i] = gth_part.sum(1)
            grho[i] = gm_part.sum((1, 2)) * ((rho[i] >= 0.0) & (rho[i] <= 1.0)).float()
            ngE = torch.empty(G, B, d, **bf)
            gemm_ops.matmul_nn(ngrb, sh[f"layer{i}.W"], ngE)  # -dE = -dr W
            t = torch.empty(G, B, n, **(bf if first else f32))
            gemm_ops.matmul_nt(ngE, Db, t)  # dy through P = y D
            wterms[i] = (ngrb, rneg_i)
            dterms.append((yb_i, ngE))
            if first:
                dterms += [(ub, xb), (t, xb)]  # dy_0 = dr_0 + dxs_0 + t_0 (xs_0 is y_0)
            gy, gy2, gx, l1c = gr, t, gxs, None
        # the weight gradients last, two problems per launch (one [n, d] problem is half the GPU's
        # 256x256 tiles), a lone problem split along K; the Adam kernel sums the split slabs
        probs = [dterms[k:k + 2] for k in range(0, len(dterms), 2)]
        dsplits = self._wg_splits([len(q) for q in probs], B)
        slabs = torch.empty(sum(dsplits), G, n, d, **f32)
        self._wg_launch(probs, dsplits, slabs)
        order = sorted(wterms, reverse=True)
        wsplits = self._wg_splits([1] * L, B)
        gW = {i: torch.empty(wsplits[k], G, n, d, **f32) for k, i in enumerate(order)}
        self._wg_launch([[wterms[i]] for i in order], wsplits, None, outs=[gW[i] for i in order])
        vec = {}
        for i in range(L):
            vec[f"layer{i}.theta"], vec[f"layer{i}.rho"] = gth[i], grho[i]
        return slabs, gW, vec, (l_rec + l_l1, l_rec, l_l1, c)

    def _wg_splits(self, nsegs, B):
        """Split-K factor per weight-gradient problem: problems run in pairs of equal segment count;
        a lone one is split so its launch still fills the GPU."""
        from ..ops import gemm as gemm_ops

        G, n, d = self.params["decoder"].shape
        out, k = [], 0
        while k < len(nsegs):
            if k + 1 < len(nsegs) and nsegs[k + 1] == nsegs[k]:
                out += [1, 1]
                k += 2
            else:
                out.append(gemm_ops.wgrad_split(G, n, d, B * nsegs[k], 1))
                k += 1
        return out

    @staticmethod
    def _wg_launch(probs, splits, slabs, outs=None):
        from ..ops import gemm as gemm_ops

        k = j = 0
        while k < len(probs):
            if splits[k] == 1 and k + 1 < len(probs) and splits[k + 1] == 1 and len(probs[k]) == len(probs[k + 1]):
                o = [slabs[j], slabs[j + 1]] if outs is None else [outs[k][0], outs[k + 1][0]]
                gemm_ops.weight_grads([probs[k], probs[k + 1]], o, 1.0, cfg=_WG_CFG)
                k, j = k + 2, j + 2
            else:
                s = splits[k]
                o = (slabs[j:j + s] if outs is None else outs[k])
                gemm_ops.weight_grads([probs[k]], [o if s > 1 else o[0]], 1.0, ksplit=s, cfg=_WG_CFG)
                k, j = k + 1, j + s

    @torch.no_grad()
    def _residual_fused_grads(self, x: torch.Tensor):
        """The residual-denoising family's step without autograd (reference
        autoencoders/residual_denoising_autoencoder.py:92-122).  Forward (c_0 = x D^T):
        h_i = relu(c_i + theta_i), c_{i+1} = h_i W_i^T + c_i, codes c = relu(c_L + b).  Backward
        (G = dL/dc_{i+1}):  dW_i = G^T h_i,  dh = G W_i,  dc_i = G + dh 1[c_i + theta_i > 0],
        dtheta_i / db = column sums of the masked terms, dD_hat = dc_0^T x + c^T dL/dx_hat."""
        from ..ops import _lib
        from ..ops import gemm as gemm_ops

        G, n, d = self.params["decoder"].shape
        B, L, dev = int(x.shape[0]), self.n_layers, self.device
        f32 = dict(device=dev, dtype=torch.float32)
        bf = dict(device=dev, dtype=torch.bfloat16)
        sh = self._shadows()
        Db = sh["decoder"]
        xb = x.to(dev, torch.bfloat16).contiguous()
        p, st = _lib.ptr, _lib.stream_handle()
        ths = [self.params[f"layer{i}.theta"].detach().contiguous() for i in range(L)]
        bias = self.params["encoder_bias"].detach().contiguous()
        part = torch.empty(G, (B // 128) * (d // 128), **f32)
        absp = torch.empty(G * B * n // 1024, **f32)

        def fwd(u, cin, th, cout, hb, fin):
            _lib.check(_lib.lib().sc_res_fwd(p(u), p(cin), p(th), p(cout), p(hb), p(absp) if fin else None, int(fin),
                                             G, B, n, st), "sc_res_fwd")

        # ---- forward
        cs, hbs = [torch.empty(G, B, n, **f32)], [torch.empty(G, B, n, **bf)]
        gemm_ops.matmul_nt(xb, Db, cs[0])  # c_0 = x D^T
        if L == 0:
            c, cb = torch.empty(G, B, n, **f32), torch.empty(G, B, n, **bf)
            fwd(None, cs[0], bias, c, cb, True)
        else:
            fwd(None, cs[0], ths[0], None, hbs[0], False)
        for i in range(L):
            u = torch.empty(G, B, n, **f32)
            gemm_ops.matmul_nt(hbs[i], sh[f"layer{i}.W"], u)  # h_i W_i^T
            if i + 1 < L:
                cs.append(torch.empty(G, B, n, **f32))
                hbs.append(torch.empty(G, B, n, **bf))
                fwd(u, cs[i], ths[i + 1], cs[i + 1], hbs[i + 1], False)
            else:
                c, cb = torch.empty(G, B, n, **f32), torch.empty(G, B, n, **bf)
                fwd(u, cs[i], bias, c, cb, True)
        rf = torch.empty(G, B, d, **bf)
        gemm_ops.decode_residual(cb, Db, xb, rf, part)
        l_rec = part.sum(1) / (B * d)
        l_l1 = self.l1 * absp.view(G, -1).sum(1) / B

        # ---- backward
        alpha = 2.0 / (B * d)
        gc = torch.empty(G, B, n, **f32)
        gemm_ops.matmul_nt(rf, Db, gc, alpha=alpha)
        rb = 64
        cpart = torch.empty(G, B // rb, n, **f32)
        vec = {}

        def bwd(gin, gadd, pre, th, l1c, out, outb):
            _lib.check(_lib.lib().sc_res_bwd(p(gin), p(gadd), p(pre), p(th), p(l1c), p(out), p(outb), p(cpart),
                                             G, B, n, rb, st), "sc_res_bwd")
            return cpart.sum(1)

        Gf, Gb = torch.empty(G, B, n, **f32), torch.empty(G, B, n, **bf)
        vec["encoder_bias"] = bwd(gc, None, c, None, (self.l1 / B).float().contiguous(), Gf, Gb)
        gW = {}
        for i in reversed(range(L)):  # (an [n, n] weight gradient is G n^2 / 256^2 >= 256 tiles: no split)
            gW[i] = torch.empty(1, G, n, n, **f32)
            gemm_ops.weight_grads([[(Gb, hbs[i])]], [gW[i][0]], 1.0, cfg=_WG_CFG)  # G^T h_i
            gh = torch.empty(G, B, n, **f32)
            gemm_ops.matmul_nn(Gb, sh[f"layer{i}.W"], gh)  # G W_i
            Gf2 = torch.empty(G, B, n, **f32) if i else None
            Gb2 = torch.empty(G, B, n, **bf)
            vec[f"layer{i}.theta"] = bwd(Gf, gh, cs[i], ths[i], None, Gf2, Gb2)
            Gf, Gb = Gf2, Gb2
        probs = [[(Gb, xb), (cb, rf.mul(alpha))]]  # dc_0^T x + c^T dL/dx_hat
        dsplits = self._wg_splits([2], B)
        slabs = torch.empty(dsplits[0], G, n, d, **f32)
        self._wg_launch(probs, dsplits, slabs)
        return slabs, gW, vec, (l_rec + l_l1, l_rec, l_l1, c)

    def fused_grads(self, x: torch.Tensor):
        """The explicit step's gradients in the autograd path's form (tests): the decoder's through
        the unit-row Jacobian, the split slabs summed."""
        slabs, gW, vec, losses = self._fused_grads(x)
        dec = self.params["decoder"].detach()
        nrm = torch.linalg.vector_norm(dec, dim=-1, keepdim=True).clamp_min(1e-8)
        gh = slabs.sum(0)
        out = {"decoder": gh / nrm - dec * (dec * gh).sum(-1, keepdim=True) / nrm ** 3}
        for i in range(self.n_layers):
            out[f"layer{i}.W"] = gW[i].sum(0)
        out.update(vec)
        return out, losses

    @torch.no_grad()
    def _fused_grads(self, x: torch.Tensor):
        return self._lista_fused_grads(x) if self.kind == "lista" else self._residual_fused_grads(x)

    @torch.no_grad()
    def _fused_step(self, x: torch.Tensor):
        from ..ops import adam as adam_ops

        slabs, gW, vec, losses = self._fused_grads(x)
        G, n, d = self.params["decoder"].shape
        sh = self._sh
        # ---- update: the row-Adam kernel (and the shadows) for the matrices, torch for the vectors
        L = self.n_layers
        self.step_count += 1
        b1, b2 = self.betas
        dec = self.params["decoder"]
        adam_ops.adam_rows([dict(p=dec.data, g=slabs[0], m=self.m["decoder"], v=self.v["decoder"],
                                 shadow=sh["decoder"], norms=None, norm=True)], self.lr, self.step_count, b1, b2,
                           self.eps, nsplit=slabs.shape[0], gstride=G * n * d)
        for i in range(L):
            k = f"layer{i}.W"
            w = self.params[k]
            adam_ops.adam_rows([dict(p=w.data, g=gW[i][0], m=self.m[k], v=self.v[k], shadow=sh[k],
                                     norms=None, norm=False)], self.lr, self.step_count, b1, b2, self.eps,
                               nsplit=gW[i].shape[0], gstride=w[0].numel() * G)
        # the vectors (theta [G, n], rho [G], the residual family's encoder bias [G, n]): torch Adam as
        # multi-tensor ops (a handful of launches)
        bc1 = 1.0 - b1 ** self.step_count
        bc2 = 1.0 - b2 ** self.step_count
        keys = list(vec)
        gs = [vec[k] for k in keys]
        ps, ms_, vs = [self.params[k].data for k in keys], [self.m[k] for k in keys], [self.v[k] for k in keys]
        torch._foreach_mul_(ms_, b1)
        torch._foreach_add_(ms_, gs, alpha=1.0 - b1)
        torch._foreach_mul_(vs, b2)
        torch._foreach_addcmul_(vs, gs, gs, value=1.0 - b2)
        den = torch._foreach_div(vs, bc2)
        torch._foreach_sqrt_(den)
        torch._foreach_add_(den, self.eps)
        upd = torch._foreach_div(ms_, den)
        lrs = [self.lr.view(-1, *([1] * (t.dim() - 1))) * (1.0 / bc1) for t in ps]
        torch._foreach_mul_(upd, [l.expand_as(u) for l, u in zip(lrs, upd)])
        torch._foreach_sub_(ps, upd)
        return losses

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
        self._sh = None
