"""Unrolled-solver encoders: LISTA and residual denoising SAEs
(reference ``autoencoders/residual_denoising_autoencoder.py:9-201``)."""

from __future__ import annotations

import torch
import torch.nn.functional as F
from torch.utils import _pytree as pytree

from .learned_dict import LearnedDict
from .signatures import DictSignature, unit_rows


def shrinkage(r, theta):
    """Soft threshold sign(r) * relu(|r| - theta)."""
    return torch.sign(r) * F.relu(r.abs() - theta)


def _orthogonal(rows, cols, dtype, device=None):
    w = torch.empty(rows, cols, dtype=dtype)
    torch.nn.init.orthogonal_(w)
    return w.to(device)


class LISTALayer:
    """One learned ISTA step with momentum (https://arxiv.org/pdf/2008.02683.pdf)."""

    @staticmethod
    def init(d_activation, n_features, dtype=torch.float32, device=None):
        return {"W": _orthogonal(n_features, d_activation, dtype, device),
                "theta": torch.randn(n_features, dtype=dtype, device=device) * 0.02,
                "rho": torch.tensor(0.1, dtype=dtype, device=device)}

    @staticmethod
    def forward(params, y, b, x, A):
        m = torch.clamp(params["rho"], 0.0, 1.0)
        r = y + (b - y @ A) @ params["W"].T
        x_ = shrinkage(r, params["theta"])
        return x_ + m * (x_ - x), x_


class FunctionalLISTADenoisingSAE(DictSignature):
    @staticmethod
    def init(d_activation, n_features, n_hidden_layers, l1_alpha, dtype=torch.float32, device=None):
        params = {"decoder": _orthogonal(n_features, d_activation, dtype, device),
                  "encoder_layers": [LISTALayer.init(d_activation, n_features, dtype, device)
                                     for _ in range(n_hidden_layers)]}
        return params, {"l1_alpha": torch.tensor(l1_alpha, dtype=dtype, device=device)}

    @staticmethod
    def encode(params, b, learned_dict):
        y = b @ learned_dict.T
        x = y
        for layer in params["encoder_layers"]:
            y, x = LISTALayer.forward(layer, y, b, x, learned_dict)
        return y

    @staticmethod
    def loss(params, buffers, batch):
        D = unit_rows(params["decoder"])
        c = FunctionalLISTADenoisingSAE.encode(params, batch, D)
        l_rec = (c @ D - batch).pow(2).mean()
        l_sp = buffers["l1_alpha"] * c.abs().sum(-1).mean()
        return l_rec + l_sp, ({"loss": l_rec + l_sp, "l_reconstruction": l_rec, "l_l1": l_sp}, {"c": c})

    @staticmethod
    def to_learned_dict(params, buffers):
        return LISTADenoisingSAE(params)

    @staticmethod
    def init_lr(n_hidden_layers, lr, lr_encoder=None):
        lr_encoder = lr if lr_encoder is None else lr_encoder
        return {"decoder": lr, "encoder_embedding": lr_encoder, "encoder_bias": lr_encoder,
                "encoder_layers": [{"weight": lr, "bias": lr} for _ in range(n_hidden_layers)]}


class LISTADenoisingSAE(LearnedDict):
    def __init__(self, params):
        self.params = params
        self.n_feats, self.activation_size = params["decoder"].shape

    def encode(self, x):
        return FunctionalLISTADenoisingSAE.encode(self.params, x, self.get_learned_dict())

    def to_device(self, device):
        self.params = pytree.tree_map(lambda t: t.to(device), self.params)

    def get_learned_dict(self):
        return unit_rows(self.params["decoder"])


class ResidualDenoisingLayer:
    @staticmethod
    def init(d_activation, n_features, dtype=torch.float32, device=None):
        return {"W": _orthogonal(n_features, n_features, dtype, device),
                "theta": torch.randn(n_features, dtype=dtype, device=device) * 0.02}

    @staticmethod
    def forward(params, x):
        return F.relu(x + params["theta"]) @ params["W"].T + x


class FunctionalResidualDenoisingSAE(DictSignature):
    @staticmethod
    def init(d_activation, n_features, n_hidden_layers, l1_alpha, dtype=torch.float32, device=None):
        params = {"decoder": _orthogonal(n_features, d_activation, dtype, device),
                  "encoder_layers": [ResidualDenoisingLayer.init(d_activation, n_features, dtype, device)
                                     for _ in range(n_hidden_layers)],
                  "encoder_bias": torch.randn(n_features, dtype=dtype, device=device) * 0.02}
        return params, {"l1_alpha": torch.tensor(l1_alpha, dtype=dtype, device=device)}

    @staticmethod
    def encode(params, b, learned_dict):
        x = b @ learned_dict.T
        for layer in params["encoder_layers"]:
            x = ResidualDenoisingLayer.forward(layer, x)
        return F.relu(x + params["encoder_bias"])

    @staticmethod
    def loss(params, buffers, batch):
        D = unit_rows(params["decoder"])
        c = FunctionalResidualDenoisingSAE.encode(params, batch, D)
        l_rec = (c @ D - batch).pow(2).mean()
        l_sp = buffers["l1_alpha"] * c.abs().sum(-1).mean()
        return l_rec + l_sp, ({"loss": l_rec + l_sp, "l_reconstruction": l_rec, "l_l1": l_sp}, {"c": c})

    @staticmethod
    def to_learned_dict(params, buffers):
        return ResidualDenoisingSAE(params)


class ResidualDenoisingSAE(LearnedDict):
    """fix B#12: reads ``params["decoder"]`` (the reference reads a missing ``"dict"`` key)."""

    def __init__(self, params):
        self.params = params
        self.n_feats, self.activation_size = params["decoder"].shape

    def encode(self, x):
        return FunctionalResidualDenoisingSAE.encode(self.params, x, self.get_learned_dict())

    def to_device(self, device):
        self.params = pytree.tree_map(lambda t: t.to(device), self.params)

    def get_learned_dict(self):
        return unit_rows(self.params["decoder"])
