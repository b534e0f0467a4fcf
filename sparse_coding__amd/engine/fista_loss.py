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
                "step": self.step_count}

    def load_state_dict(self, st):
        with torch.no_grad():
            for k, v in st["params"].items():
                self.params[k].copy_(v)
        self.opt.load_state_dict(st["optim"])
        self.step_count = int(st["step"])
