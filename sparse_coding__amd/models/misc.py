"""Remaining dictionary learners of the reference:

* ``SemiLinearSAE`` -- 2-layer ReLU MLP encoder + normalised decoder
  (reference ``autoencoders/semilinear_autoencoder.py:31-83``); fix B#29: gains a
  ``to_learned_dict`` (``SemiLinearDict``) so sweeps can checkpoint it.
* Positive SAEs -- non-negative tied dictionary with a +0.18 input shift
  (reference ``autoencoders/mlp_tests.py:8-125``).
* ``RICA`` -- reconstruction ICA with a smooth-L1 sparsity penalty (``autoencoders/rica.py``).
* ``DirectCoefOptimizer`` / ``DirectCoefSearch`` -- basis pursuit by 100 SGD-momentum
  steps on the codes (``autoencoders/direct_coef_search.py``; fix B#8: the missing
  ``optimizers.sgdm`` dependency is replaced by an inline momentum step).
"""

from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.utils import _pytree as pytree

from .learned_dict import LearnedDict, TiedSAE
from .signatures import DictSignature, unit_rows, xavier


# ----------------------------------------------------------------- semi-linear
class FFLayer:
    @staticmethod
    def init(input_size, output_size, device=None, dtype=None):
        return {"weight": xavier((output_size, input_size), device, dtype),
                "bias": torch.zeros(output_size, device=device, dtype=dtype or torch.float32)}

    @staticmethod
    def forward(params, x):
        return torch.clamp(x @ params["weight"].T + params["bias"], min=0.0)


class SemiLinearSAE(DictSignature):
    @staticmethod
    def init(activation_size, n_dict_components, l1_alpha, device=None, dtype=None, hidden_size=None):
        hidden = hidden_size or n_dict_components
        params = {"encoder_layers": [FFLayer.init(activation_size, hidden, device, dtype),
                                     FFLayer.init(hidden, n_dict_components, device, dtype)],
                  "decoder": xavier((n_dict_components, activation_size), device, dtype)}
        return params, {"l1_alpha": torch.tensor(l1_alpha, device=device, dtype=dtype or torch.float32)}

    @staticmethod
    def encode(params, batch):
        c = batch
        for layer in params["encoder_layers"]:
            c = FFLayer.forward(layer, c)
        return c

    @staticmethod
    def loss(params, buffers, batch):
        c = SemiLinearSAE.encode(params, batch)
        x_hat = c @ unit_rows(params["decoder"])
        l_rec = (x_hat - batch).pow(2).mean()
        l_l1 = buffers["l1_alpha"] * c.abs().sum(-1).mean()
        return l_rec + l_l1, ({"loss": l_rec + l_l1, "l_reconstruction": l_rec, "l_l1": l_l1}, {"c": c})

    @staticmethod
    def to_learned_dict(params, buffers):
        return SemiLinearDict(params)


class SemiLinearDict(LearnedDict):
    def __init__(self, params):
        self.params = params
        self.n_feats, self.activation_size = params["decoder"].shape

    def encode(self, batch):
        return SemiLinearSAE.encode(self.params, batch)

    def get_learned_dict(self):
        return unit_rows(self.params["decoder"])

    def to_device(self, device):
        self.params = pytree.tree_map(lambda t: t.to(device), self.params)


# ----------------------------------------------------------------- positive SAEs
POSITIVE_SHIFT = 0.18


class TiedPositiveSAE(LearnedDict):
    """fix B#20: no stray ``encoder.clamp`` attribute; the encoder is clamped >= 0 on use."""

    def __init__(self, encoder, encoder_bias, norm_encoder=False):
        self.encoder = encoder.abs()
        self.encoder_bias = encoder_bias
        self.norm_encoder = norm_encoder
        self.n_feats, self.activation_size = self.encoder.shape

    def get_learned_dict(self):
        return unit_rows(self.encoder)

    def to_device(self, device):
        self.encoder = self.encoder.to(device)
        self.encoder_bias = self.encoder_bias.to(device)

    def encode(self, batch):
        enc = torch.clamp(self.encoder, min=0.0)
        enc = unit_rows(enc) if self.norm_encoder else enc
        return torch.clamp(batch @ enc.T + self.encoder_bias, min=0.0)


class UntiedPositiveSAE(TiedPositiveSAE):
    """fix B#20: uses its (optionally normalised) encoder for encoding."""

    def __init__(self, encoder, encoder_bias, decoder, norm_encoder=False):
        super().__init__(encoder, encoder_bias, norm_encoder)
        self.decoder = decoder

    def to_device(self, device):
        super().to_device(device)
        self.decoder = self.decoder.to(device)


class FunctionalPositiveTiedSAE(DictSignature):
    @staticmethod
    def init(activation_size, n_dict_components, l1_alpha, bias_decay=0.0, device=None, dtype=None):
        dt = dtype or torch.float32
        params = {"encoder": xavier((n_dict_components, activation_size), device, dtype).abs(),
                  "encoder_bias": torch.full((n_dict_components,), -1.0, device=device, dtype=dt)}
        buffers = {"l1_alpha": torch.tensor(l1_alpha, device=device, dtype=dt),
                   "bias_decay": torch.tensor(bias_decay, device=device, dtype=dt)}
        return params, buffers

    @staticmethod
    def to_learned_dict(params, buffers):
        return TiedSAE(torch.clamp(params["encoder"], min=0.0), params["encoder_bias"], norm_encoder=True)

    @staticmethod
    def loss(params, buffers, batch):
        w = unit_rows(torch.clamp(params["encoder"], min=0.0))
        c = torch.clamp((batch + POSITIVE_SHIFT) @ w.T + params["encoder_bias"], min=0.0)
        x_hat = c @ w
        l_rec = ((x_hat - POSITIVE_SHIFT) - batch).pow(2).mean()
        l_l1 = buffers["l1_alpha"] * c.abs().sum(-1).mean()
        l_bd = buffers["bias_decay"] * torch.linalg.vector_norm(params["encoder_bias"])
        total = l_rec + l_l1 + l_bd
        return total, ({"loss": total, "l_reconstruction": l_rec, "l_l1": l_l1, "l_bias_decay": l_bd}, {"c": c})


# ----------------------------------------------------------------- RICA
class RICA(nn.Module):
    """Reconstruction ICA (Le et al.); fix: calls ``nn.Module.__init__``."""

    def __init__(self, activation_size, n_dict_components, sparsity_coef=0.0, sparsity_loss="smooth_l1"):
        super().__init__()
        self.n_dict_components = n_dict_components
        self.activation_size = activation_size
        self.weights = nn.Parameter(xavier((n_dict_components, activation_size)))
        self.sparsity_loss = sparsity_loss
        self.sparsity_coef = sparsity_coef

    def forward(self, x):
        c = x @ self.weights.T
        return c @ self.weights, c

    def loss(self, x, x_hat, c):
        l_rec = F.mse_loss(x, x_hat)
        if self.sparsity_loss == "smooth_l1":
            l_sp = F.smooth_l1_loss(c, torch.zeros_like(c))
        elif self.sparsity_loss == "l1":
            l_sp = F.l1_loss(c, torch.zeros_like(c))
        else:
            raise ValueError(self.sparsity_loss)
        return l_rec + self.sparsity_coef * l_sp, l_rec, l_sp

    def train_batch(self, batch, optimizer=None):
        if optimizer is None:
            raise ValueError("optimizer must be specified for RICA")
        optimizer.zero_grad()
        x_hat, c = self(batch)
        loss, l_rec, l_sp = self.loss(batch, x_hat, c)
        loss.backward()
        optimizer.step()
        return loss.detach(), l_rec.detach(), l_sp.detach()

    def get_dict(self):
        return self.weights

    def configure_optimizers(self, **kwargs):
        return torch.optim.Adam(self.parameters(), **kwargs)


# ----------------------------------------------------------------- direct coefficient search
N_ITERS_OPT = 100


class DirectCoefOptimizer(DictSignature):
    @staticmethod
    def init(d_activation, n_features, l1_alpha, lr=1e-3, dtype=torch.float32, device=None):
        params = {"decoder": torch.randn(n_features, d_activation, dtype=dtype, device=device)}
        buffers = {"l1_alpha": torch.tensor(l1_alpha, dtype=dtype, device=device),
                   "lr": torch.tensor(lr, dtype=dtype, device=device)}
        return params, buffers

    @staticmethod
    def objective(c, normed_dict, batch, l1_alpha):
        l_rec = (c @ normed_dict - batch).pow(2).mean()
        l_sp = l1_alpha * c.abs().sum(-1).mean()
        return l_rec + l_sp, ({"loss": l_rec + l_sp, "l_reconstruction": l_rec, "l_l1": l_sp}, {"c": c})

    @staticmethod
    def basis_pursuit(params, buffers, batch, normed_dict=None, n_iters=N_ITERS_OPT, momentum=0.9):
        """Projected SGD with momentum on the codes (closed-form gradient of the objective).
        On the GPU (outside autograd / vmap, supported shapes) this is the persistent HIP
        solver's coefficient-search mode (``ops.fista.coef_search``)."""
        D = unit_rows(params["decoder"]) if normed_dict is None else normed_dict
        B, d = batch.shape
        if batch.is_cuda and not torch._C._functorch.is_functorch_wrapped_tensor(batch) \
                and not torch.is_grad_enabled():
            from ..ops import fista as fista_ops

            try:
                return fista_ops.coef_search(batch, D.detach()[None], buffers["l1_alpha"], buffers["lr"], n_iters,
                                             momentum, backend="auto")[0].to(batch.dtype)
            except ValueError:
                pass
        c = torch.zeros(B, D.shape[0], device=batch.device, dtype=batch.dtype)
        buf = torch.zeros_like(c)
        lr, lam = buffers["lr"], buffers["l1_alpha"]
        for _ in range(n_iters):
            grad = 2.0 / (B * d) * (c @ D - batch) @ D.T + lam / B * torch.sign(c)
            buf = momentum * buf + grad
            c = F.relu(c - lr * buf)
        return c

    @staticmethod
    def loss(params, buffers, batch):
        D = unit_rows(params["decoder"])
        with torch.no_grad():
            c = DirectCoefOptimizer.basis_pursuit(params, buffers, batch, normed_dict=D)
        l_rec = (c @ D - batch).pow(2).mean()
        return l_rec, ({"loss": l_rec}, {"c": c})

    @staticmethod
    def to_learned_dict(params, buffers):
        return DirectCoefSearch(params, buffers)


class DirectCoefSearch(LearnedDict):
    def __init__(self, params, buffers):
        self.params = params
        self.buffers = buffers
        self.n_feats, self.activation_size = params["decoder"].shape

    def encode(self, x):
        return DirectCoefOptimizer.basis_pursuit(self.params, self.buffers, x)

    def get_learned_dict(self):
        return unit_rows(self.params["decoder"])

    def to_device(self, device):
        self.params = pytree.tree_map(lambda t: t.to(device), self.params)
        self.buffers = pytree.tree_map(lambda t: t.to(device), self.buffers)
