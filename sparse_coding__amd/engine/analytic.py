"""Closed-form SAE ensemble step in plain PyTorch (CPU fast path, second oracle).

The reference differentiates each model's loss with ``vmap(grad(loss))`` and applies
torchopt Adam (``autoencoders/ensemble.py:119-123, 175-193``).  For the SAE family the
gradients have a short closed form -- the same algebra the gfx950
kernels implement -- so this engine evaluates it with batched GEMMs on the stacked
parameters: no autograd graph, no vmap dispatch.  On the CPU (BASELINE config 1) this
is several times faster than the transform-based path; it is exact in fp32.

    x_c   = center(x)                       (tied: fixed affine buffers; untied: x)
    w_hat = W / max(|W|_row, 1e-8)
    pre   = x_c W_e^T + b,  c = relu(pre) (masked features forced to 0)
    R     = c W_hat_d - x_c
    L     = mean(R^2) + l1 * mean_b |c|_1 + bias_decay * |b|
    G     = 2 R / (B d)
    dpre  = 1[pre >= 0] (G W_hat_d^T + l1 / B)
    dW_hat_d = c^T G    (tied: + dpre^T x_c)
    dW    = (dW_hat - w_hat <w_hat, dW_hat>) / |W|     (|W| <= 1e-8: dW_hat / 1e-8)
    dW_e  = dpre^T x_c  (untied),   db = sum_b dpre + bias_decay * b / |b|
"""

from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch

from ..models.signatures import (FunctionalMaskedSAE, FunctionalMaskedTiedSAE, FunctionalSAE, FunctionalTiedSAE,
                                 unit_rows)

_KINDS = {FunctionalSAE: "untied", FunctionalMaskedSAE: "untied", FunctionalTiedSAE: "tied",
          FunctionalMaskedTiedSAE: "tied"}
FLOOR = 1e-8


def supports(sig) -> bool:
    from ..models.fista import FunctionalFista

    return sig in _KINDS or sig is FunctionalFista


def _norm_backward(w: torch.Tensor, w_hat: torch.Tensor, g_hat: torch.Tensor) -> torch.Tensor:
    nrm = torch.linalg.vector_norm(w, dim=-1, keepdim=True)
    big = nrm > FLOOR
    proj = g_hat - w_hat * (w_hat * g_hat).sum(-1, keepdim=True)
    return torch.where(big, proj / nrm.clamp(min=FLOOR), g_hat / FLOOR)


class AnalyticSAEEnsemble:
    def __init__(self, models: List[Tuple[dict, dict]], sig, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 device="cpu"):
        from ..models.fista import FunctionalFista

        self.sig = sig
        self.kind = "untied" if sig is FunctionalFista else _KINDS[sig]
        self.device = torch.device(device)
        self.n_models = len(models)

        def stack(key, src=0):
            return torch.stack([m[src][key].detach().to(self.device, torch.float32) for m in models]).contiguous()

        self.params: Dict[str, torch.Tensor] = {"encoder": stack("encoder"), "encoder_bias": stack("encoder_bias")}
        if self.kind == "untied":
            self.params["decoder"] = stack("decoder")
        b0 = models[0][1]
        self.buffers = {k: torch.stack([m[1][k].to(self.device) for m in models]) for k in b0}
        G, n, d = self.params["encoder"].shape
        self.n, self.d = n, d
        self.l1 = self.buffers["l1_alpha"].float().reshape(G)
        self.bias_decay = self.buffers.get("bias_decay", torch.zeros(G, device=self.device)).float().reshape(G)
        self.live = None
        self.masked = "coef_mask" in self.buffers
        if self.masked:  # masked signatures have no bias-decay term in their loss
            self.bias_decay = torch.zeros_like(self.bias_decay)
            self.live = (~self.buffers["coef_mask"].bool()).float().reshape(G, 1, n)
        self.identity_center = True
        if "center_rot" in self.buffers:
            bf = self.buffers
            eye = torch.eye(d, device=self.device).expand_as(bf["center_rot"])
            self.identity_center = bool(torch.equal(bf["center_rot"].float(), eye)
                                        and not bf["center_trans"].any() and bool((bf["center_scale"] == 1).all()))
        self.lr, self.betas, self.eps = lr, betas, eps
        self.m = {k: torch.zeros_like(v) for k, v in self.params.items()}
        self.v = {k: torch.zeros_like(v) for k, v in self.params.items()}
        self.count = 0
        self.last_losses: Dict[str, torch.Tensor] = {}
        self.last_codes: Optional[torch.Tensor] = None

    # ------------------------------------------------------------------ math
    def _center(self, x):
        if self.kind == "tied" and not self.identity_center:
            bf = self.buffers
            xc = (x.unsqueeze(0) - bf["center_trans"].unsqueeze(1)) @ bf["center_rot"].transpose(-1, -2)
            return xc * bf["center_scale"].unsqueeze(1)
        return x.unsqueeze(0).expand(self.n_models, *x.shape)

    def compute_grads(self, x: torch.Tensor):
        P = self.params
        G, n, d = P["encoder"].shape
        x = x.to(self.device, torch.float32)
        B = x.shape[-2]
        xc = self._center(x) if x.dim() == 2 else x
        w_e = P["encoder"]
        if self.kind == "tied":
            w_e = unit_rows(w_e)
            w_d = w_e
        else:
            w_d = unit_rows(P["decoder"])
        pre = torch.baddbmm(P["encoder_bias"].unsqueeze(1), xc, w_e.transpose(1, 2))
        c = pre.clamp(min=0.0)
        if self.live is not None:
            c = c * self.live
        R = torch.bmm(c, w_d) - xc
        l1 = self.l1.view(G, 1, 1)
        bnorm = torch.linalg.vector_norm(P["encoder_bias"], dim=-1)
        l_rec = R.pow(2).mean(dim=(1, 2))
        l_l1 = self.l1 * c.sum(-1).mean(-1)
        l_bd = self.bias_decay * bnorm
        Gm = R * (2.0 / (B * d))
        dc = torch.bmm(Gm, w_d.transpose(1, 2)) + l1 / B
        dpre = dc * (pre >= 0).float()
        if self.live is not None:
            dpre = dpre * self.live
        grads = {}
        g_hat_d = torch.bmm(c.transpose(1, 2), Gm)
        if self.kind == "tied":
            g_hat = g_hat_d + torch.bmm(dpre.transpose(1, 2), xc)
            grads["encoder"] = _norm_backward(P["encoder"], w_e, g_hat)
        else:
            grads["decoder"] = _norm_backward(P["decoder"], w_d, g_hat_d)
            grads["encoder"] = torch.bmm(dpre.transpose(1, 2), xc)
        db = dpre.sum(1)
        db = db + torch.where(bnorm.unsqueeze(-1) > 0, P["encoder_bias"] / bnorm.clamp(min=1e-30).unsqueeze(-1),
                              torch.zeros_like(db)) * self.bias_decay.unsqueeze(-1)
        grads["encoder_bias"] = db
        losses = {"loss": l_rec + l_l1 + l_bd, "l_reconstruction": l_rec, "l_l1": l_l1}
        if self.kind == "untied" and not self.masked:
            losses["l_bias_decay"] = l_bd
        self.last_losses = losses
        self.last_codes = c
        return grads, (losses, {"c": c})

    def apply_grads(self, grads):
        self.count += 1
        b1, b2 = self.betas
        bc1 = 1 - b1 ** self.count
        bc2 = 1 - b2 ** self.count
        for k, g in grads.items():
            m, v = self.m[k], self.v[k]
            m.mul_(b1).add_(g, alpha=1 - b1)
            v.mul_(b2).addcmul_(g, g, value=1 - b2)
            self.params[k].addcdiv_(m, (v / bc2).sqrt_().add_(self.eps), value=-self.lr / bc1)

    def step_batch(self, x):
        grads, (losses, aux) = self.compute_grads(x)
        self.apply_grads(grads)
        return losses, aux

    # ------------------------------------------------------------------ export / state
    def unstack(self, device="cpu"):
        out = []
        for g in range(self.n_models):
            p = {k: v[g].detach().to(device).clone() for k, v in self.params.items()}
            b = {k: v[g].detach().to(device).clone() for k, v in self.buffers.items()}
            out.append((p, b))
        return out

    def to_learned_dicts(self, device="cpu"):
        return [self.sig.to_learned_dict(p, b) for p, b in self.unstack(device)]

    def state_dict(self):
        return {"params": self.params, "m": self.m, "v": self.v, "count": self.count}

    def load_state_dict(self, sd):
        for d_ in ("params", "m", "v"):
            for k, t in sd[d_].items():
                getattr(self, d_)[k].copy_(t)
        self.count = int(sd["count"])
