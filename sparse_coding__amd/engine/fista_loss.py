"""``FistaLossEnsemble``: the "FISTA in the loss" objective (reference
``autoencoders/fista.py:141-172``, the fork's fista_13_10 runs) for a whole L1 sweep at once.

Per model (stacked over G): w = unit_rows(encoder), c = relu(x w^T + b),
    loss = |c w - x|^2 / (B d) + l1 |c|_1 / B + bias_decay |b| + |x - FISTA_T(c; w) w|^2 / (B d)
where FISTA_T is T unrolled iterations warm-started at c.  The T-iteration solve and its
adjoint run on the kernels (``ops.fista.unrolled_fista_residual``: direct-form HIP solver
saving the bf16 iterate slabs, adjoint sweep of grouped MFMA GEMMs + one elementwise kernel
per iteration, one K = T B GEMM for the dictionary gradient); eta = 1 / lambda_max(w w^T)
per model comes from the warm ``EtaTracker`` (power iteration, exact refresh every 50
calls) instead of an eigvalsh per call, and -- like the reference's undetached eigvalsh --
carries its gradient (d lambda_max / dw = 2 (w u) u^T, ``ops.fista.tracked_eta``).  The rest of the graph (two bmm, the norms) is
ordinary autograd, and Adam is torch's fused multi-tensor Adam over the stacked tensors
(elementwise, so per-model exact).
"""

from __future__ import annotations

import torch

from ..ops import fista as fista_ops


def fused_ok(models, batch_size: int, device, num_iter: int):
    """Whether ``FusedFistaLossEnsemble`` runs these models: GPU kernels present, the fused
    tied-SAE shapes (B % 128, n % 128, d % 256) and the Gram FISTA kernel (n in GRAM_N, n <= d)."""
    from ..ops import _lib

    dev = torch.device(device)
    n, d = models[0][0]["encoder"].shape
    if dev.type != "cuda" or not _lib.available():
        return False
    return (batch_size % 128 == 0 and n % 128 == 0 and d % 256 == 0 and n in fista_ops.GRAM_N and n <= d
            and num_iter >= 1)


class FistaLossEnsemble:
    def __init__(self, models, lr: float = 1e-3, batch_size: int = 256, device="cuda", num_iter: int = 50,
                 backend: str = "auto", betas=(0.9, 0.999), eps: float = 1e-8):
        self.device = dev = torch.device(device)
        self.n_models = G = len(models)
        self.batch_size = int(batch_size)
        self.num_iter = int(num_iter)
        self.backend = backend
        enc = torch.stack([m[0]["encoder"].detach().float() for m in models]).to(dev)
        bias = torch.stack([m[0]["encoder_bias"].detach().float() for m in models]).to(dev)
        self.params = {"encoder": enc.requires_grad_(), "encoder_bias": bias.requires_grad_()}
        self.l1 = torch.tensor([float(m[1]["l1_alpha"]) for m in models], device=dev)
        self.bias_decay = torch.tensor([float(m[1].get("bias_decay", 0.0)) for m in models], device=dev)
        self.meta = [dict(m[1]) for m in models]
        self.opt = torch.optim.Adam(list(self.params.values()), lr=lr, betas=betas, eps=eps,
                                    foreach=not dev.type == "cuda", fused=dev.type == "cuda")
        self.eta = fista_ops.EtaTracker()
        self.last = {}
        self.step_count = 0
        del G

    def losses(self, x):
        enc, b = self.params["encoder"], self.params["encoder_bias"]
        B, d = x.shape
        w = enc / enc.norm(dim=-1, keepdim=True).clamp_min(1e-8)
        c = torch.relu(torch.einsum("bd,gnd->gbn", x, w) + b[:, None, :])
        l_rec = (torch.bmm(c, w) - x).pow(2).mean(dim=(1, 2))
        l_l1 = self.l1 * c.abs().sum(-1).mean(-1)
        l_bd = self.bias_decay * b.norm(dim=-1)
        # eta = 1/lambda_max(w w^T) is differentiable in w, as in the reference (not detached)
        eta = fista_ops.tracked_eta(w, self.eta)
        R = fista_ops.unrolled_fista_residual(x, w, self.l1, c, self.num_iter, eta, backend=self.backend)
        l_fista = R.pow(2).mean(dim=(1, 2))
        return l_rec + l_fista + l_l1 + l_bd, {"l_reconstruction": l_rec, "l_fista": l_fista, "l_l1": l_l1}

    def step_batch(self, batch):
        x = batch.to(self.device, torch.float32)
        total, parts = self.losses(x)
        self.opt.zero_grad(set_to_none=True)
        total.sum().backward()  # models are independent: the sum's gradient is each model's own
        self.opt.step()
        self.step_count += 1
        self.last = {k: v.detach() for k, v in parts.items()}
        return total.detach()

    def unstack(self, device="cpu"):
        return [({k: v[i].detach().to(device).clone() for k, v in self.params.items()},
                 {k: (v.detach().to(device).clone() if torch.is_tensor(v) else v) for k, v in self.meta[i].items()})
                for i in range(self.n_models)]

    def to_learned_dicts(self, device="cpu"):
        """The trained objective is a tied SAE with row-normalised dictionary (reference
        FunctionalFista.loss2 normalises the encoder rows)."""
        from ..models.learned_dict import TiedSAE

        return [TiedSAE(p["encoder"], p["encoder_bias"], norm_encoder=True) for p, _ in self.unstack(device)]

    def state_dict(self):
        return {"params": {k: v.detach().clone() for k, v in self.params.items()}, "optim": self.opt.state_dict(),
                "step": self.step_count, "eta": self.eta.state_dict()}

    def load_state_dict(self, st):
        with torch.no_grad():
            for k, v in st["params"].items():
                self.params[k].copy_(v)
        self.opt.load_state_dict(st["optim"])
        self.step_count = int(st["step"])
        if "eta" in st:
            self.eta.load_state_dict(st["eta"])


class FusedFistaLossEnsemble:
    """FISTA in the loss entirely on the kernels (MI355X path of ``FistaLossEnsemble``).

    The tied normalised SAE half runs on the fused engine's tied kernels
    (``engine/fused.py``: encoder / decoder / code-gradient epilogues, one weight-gradient GEMM,
    row Adam with the norm Jacobian, bias Adam + loss reduction).  The unrolled FISTA term runs
    in the Gram-form kernel twice -- the T-iteration solve warm-started at the SAE codes (saving
    the bf16 Y / A slabs) and the reverse adjoint sweep -- and its gradients join the SAE's in
    the engine's own buffers before the one Adam step:

    * warm-start gradient cbar: added to the code gradient under the ReLU mask (so it reaches
      the encoder through the same weight-gradient GEMM and the bias through its column sum);
    * dictionary gradient Dbar = eta (Vsum^T X - (M + M^T) D) - A_T^T Rbar (ops/fista.py);
    * eta gradient (eta = 1 / lambda_max(w w^T), undetached as in the reference): the rank-one
      term -2 etabar eta^2 (w u) u^T with u from the warm power-iteration tracker.

    Reference: autoencoders/fista.py:141-172 (loss2); per model the objective is
    |c w - x|^2 / (B d) + l1 |c|_1 / B + bias_decay |b| + |x - FISTA_T(c; w) w|^2 / (B d)."""

    def __init__(self, models, lr: float = 1e-3, batch_size: int = 256, device="cuda", num_iter: int = 50,
                 betas=(0.9, 0.999), eps: float = 1e-8):
        from ..models.signatures import FunctionalTiedSAE
        from .fused import FusedSAEEnsemble

        self.device = torch.device(device)
        self.n_models = G = len(models)
        self.batch_size = B = int(batch_size)
        self.num_iter = T = int(num_iter)
        if not fused_ok(models, B, device, T):
            raise ValueError("fused FISTA-in-loss needs the GPU kernels, B % 128 == 0, d % 256 == 0 and n in "
                             f"{fista_ops.GRAM_N} with n <= d")
        tied = [({"encoder": p["encoder"], "encoder_bias": p["encoder_bias"]},
                 {"l1_alpha": b["l1_alpha"], "bias_decay": b.get("bias_decay", 0.0)}) for p, b in models]
        self.engine = FusedSAEEnsemble(tied, FunctionalTiedSAE, lr=lr, batch_size=B, device=device, betas=betas,
                                       eps=eps, kind="tied", track_feature_counts=False, wgrad_split=1,
                                       grad_dtype="fp32")
        self.params = self.engine.params
        self.meta = [dict(m[1]) for m in models]
        self._untouched = [{k: v.detach() for k, v in m[0].items() if k not in ("encoder", "encoder_bias")}
                           for m in models]
        self.l1 = self.engine.l1
        self.mom = fista_ops.momentum_schedule(max(T, 1))
        self._mom_list = self.mom.tolist()
        self.eta = fista_ops.EtaTracker()
        self.alpha = 2.0 / (B * self.engine.d)
        self.last = {}
        self.step_count = 0
        self.l_fista = torch.zeros(G, device=self.device)

    def compute_grads(self, batch):
        """Every gradient of the step into the engine's buffers (dictionary: ``engine.g_dec``
        w.r.t. the normalised rows, bias: ``engine.g_bias``); no update."""
        e = self.engine
        x = e._x_bf16(batch)
        a = self.alpha
        e.forward(x)
        w_f = e.params["encoder"] / e.norms.unsqueeze(-1)          # fp32 normalised rows
        eta = self.eta(w_f)
        u = self.eta.v                                               # [G, d, 1] top right singular vector
        R, st = fista_ops.unrolled_forward_gram(x, e.enc_shadow, e.c.float(), self.l1, eta.contiguous(),
                                                 self.num_iter, self.mom)
        torch.mul(R.square().mean(dim=(1, 2)), 1.0, out=self.l_fista)
        Dbar, cbar, etabar = fista_ops.unrolled_backward_gram(R.mul_(a), st, eta.contiguous(), self._mom_list,
                                                              self.num_iter, lam=self.l1)
        # warm-start gradient through the ReLU: code gradient (engine units: dL/dpre = alpha dpre)
        cm = torch.where(e.c > 0, cbar, 0.0)
        e.dpre.add_(cm, alpha=1.0 / a)
        e.backward_weights(x)
        e.g_dec.add_(Dbar)
        # eta = 1 / lambda_max(w w^T): d eta / d w = -2 eta^2 (w u) u^T
        scale = (-2.0 * etabar * eta * eta)[:, None, None]
        e.g_dec.add_(scale * torch.bmm(torch.bmm(w_f, u), u.transpose(1, 2)))
        torch.sum(e.colpart, dim=1, keepdim=True, out=e.g_bias)
        e.g_bias.mul_(a).add_(cm.sum(dim=1, keepdim=True))
        return x

    def apply_update(self):
        e = self.engine
        e.adam_rows_all()
        e._bias_loss(update=True, reduced=True)
        e._host_step()

    def step_batch(self, batch):
        self.compute_grads(batch)
        self.apply_update()
        self.step_count += 1
        out = self.engine.out
        total = out[:, 0] + self.l_fista
        self.last = {"l_reconstruction": out[:, 1], "l_fista": self.l_fista, "l_l1": out[:, 2]}
        return total

    def unstack(self, device="cpu"):
        res = []
        for i in range(self.n_models):
            p = {k: v[i].detach().to(device).clone() for k, v in self.params.items()}
            p.update({k: v.to(device).clone() for k, v in self._untouched[i].items()})
            res.append((p, {k: (v.detach().to(device).clone() if torch.is_tensor(v) else v)
                            for k, v in self.meta[i].items()}))
        return res

    def to_learned_dicts(self, device="cpu"):
        from ..models.learned_dict import TiedSAE

        return [TiedSAE(p["encoder"], p["encoder_bias"], norm_encoder=True) for p, _ in self.unstack(device)]

    def state_dict(self):
        """Masters, Adam moments, step counters (host and device) of the kernel engine, plus this
        objective's own step count and the warm power-iteration state of the eta tracker."""
        return {"engine": self.engine.state_dict(), "step": self.step_count, "eta": self.eta.state_dict()}

    def load_state_dict(self, st):
        self.engine.load_state_dict(st["engine"])  # also rebuilds the bf16 shadows and row norms
        self.step_count = int(st["step"])
        self.eta.load_state_dict(st["eta"])
