"""Functional dictionary-learner signatures (pure torch; the CPU / correctness oracle).

A *signature* is a stateless class with static methods (reference
``autoencoders/ensemble.py:15-22`` ``DictSignature``):

* ``init(...) -> (params, buffers)``  -- dicts of tensors for ONE model;
* ``loss(params, buffers, batch) -> (loss, (loss_dict, aux_dict))`` -- differentiable
  w.r.t. ``params`` so ``torch.func.grad`` / ``vmap`` can batch many models;
* ``to_learned_dict(params, buffers) -> LearnedDict``.

The math is the reference's; the fused HIP engine in
``sparse_coding__amd.engine.fused`` implements the same losses and is tested
against these functions.
"""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .learned_dict import LearnedDict, ReverseSAE, TiedSAE, UntiedSAE


class DictSignature:
    """Protocol marker (reference autoencoders/ensemble.py:15-22)."""

    @staticmethod
    def init(*args, **kwargs):
        raise NotImplementedError

    @staticmethod
    def loss(params, buffers, batch):
        raise NotImplementedError

    @staticmethod
    def to_learned_dict(params, buffers):
        raise NotImplementedError


# --------------------------------------------------------------------------- helpers
def xavier(shape, device=None, dtype=None, generator=None):
    """``nn.init.xavier_uniform_`` for a 2-D ``[fan_out, fan_in]`` weight."""
    fan_out, fan_in = shape
    a = math.sqrt(6.0 / (fan_in + fan_out))
    w = torch.empty(shape, device=device, dtype=dtype or torch.float32)
    if generator is None:
        w.uniform_(-a, a)
    else:
        w.copy_(torch.rand(shape, generator=generator, dtype=w.dtype).to(w.device) * (2 * a) - a)
    return w


def unit_rows(w: torch.Tensor, floor: float = 1e-8) -> torch.Tensor:
    return w / torch.clamp(torch.linalg.vector_norm(w, dim=-1), min=floor).unsqueeze(-1)


def relu_code(x, w, b):
    return torch.clamp(x @ w.transpose(-1, -2) + b, min=0.0)


def _scalar(v, device, dtype):
    return torch.tensor(v, device=device, dtype=dtype or torch.float32)


def _sae_losses(x_hat, x, c, l1_alpha, bias_term=None):
    l_rec = (x_hat - x).pow(2).mean()
    l_l1 = l1_alpha * c.abs().sum(dim=-1).mean()
    out = {"l_reconstruction": l_rec, "l_l1": l_l1}
    total = l_rec + l_l1
    if bias_term is not None:
        out["l_bias_decay"] = bias_term
        total = total + bias_term
    out = {"loss": total, **out}
    return total, out


# --------------------------------------------------------------------------- untied
class FunctionalSAE(DictSignature):
    """Untied SAE: ``c = relu(W_e x + b)``, ``x_hat = c W_hat``, decoder normalised in the loss.

    Reference ``autoencoders/sae_ensemble.py:13-77``.
    """

    fused_kind = "untied"

    @staticmethod
    def init(activation_size, n_dict_components, l1_alpha, bias_decay=0.0, device=None, dtype=None):
        params = {
            "encoder": xavier((n_dict_components, activation_size), device, dtype),
            "encoder_bias": torch.zeros(n_dict_components, device=device, dtype=dtype or torch.float32),
            "decoder": xavier((n_dict_components, activation_size), device, dtype),
        }
        buffers = {
            "l1_alpha": _scalar(l1_alpha, device, dtype),
            "bias_decay": _scalar(bias_decay, device, dtype),
        }
        return params, buffers

    @staticmethod
    def to_learned_dict(params, buffers):
        return UntiedSAE(params["encoder"], params["decoder"], params["encoder_bias"])

    @staticmethod
    def encode(params, buffers, batch):
        return relu_code(batch, params["encoder"], params["encoder_bias"])

    @staticmethod
    def loss(params, buffers, batch):
        c = relu_code(batch, params["encoder"], params["encoder_bias"])
        x_hat = c @ unit_rows(params["decoder"])
        bd = buffers["bias_decay"] * torch.linalg.vector_norm(params["encoder_bias"])
        total, ld = _sae_losses(x_hat, batch, c, buffers["l1_alpha"], bd)
        return total, (ld, {"c": c})


# --------------------------------------------------------------------------- tied
def _affine_center(buffers, x):
    return ((x - buffers["center_trans"]) @ buffers["center_rot"].transpose(-1, -2)) * buffers["center_scale"]


def _affine_uncenter(buffers, y):
    return (y / buffers["center_scale"]) @ buffers["center_rot"] + buffers["center_trans"]


class FunctionalTiedSAE(DictSignature):
    """Tied SAE with fixed affine centering buffers (reference sae_ensemble.py:80-160)."""

    fused_kind = "tied"

    @staticmethod
    def init(activation_size, n_dict_components, l1_alpha, device=None, dtype=None, bias_decay=0.0,
             translation=None, rotation=None, scaling=None):
        dt = dtype or torch.float32
        buffers = {
            "center_rot": rotation if rotation is not None else torch.eye(activation_size, device=device, dtype=dt),
            "center_trans": translation if translation is not None else torch.zeros(activation_size, device=device, dtype=dt),
            "center_scale": scaling if scaling is not None else torch.ones(activation_size, device=device, dtype=dt),
            "l1_alpha": _scalar(l1_alpha, device, dtype),
            "bias_decay": _scalar(bias_decay, device, dtype),
        }
        params = {
            "encoder": xavier((n_dict_components, activation_size), device, dtype),
            "encoder_bias": torch.zeros(n_dict_components, device=device, dtype=dt),
        }
        return params, buffers

    @staticmethod
    def to_learned_dict(params, buffers):
        return TiedSAE(params["encoder"], params["encoder_bias"],
                       centering=(buffers["center_trans"], buffers["center_rot"], buffers["center_scale"]),
                       norm_encoder=True)

    center = staticmethod(_affine_center)
    uncenter = staticmethod(_affine_uncenter)

    @staticmethod
    def loss(params, buffers, batch):
        w = unit_rows(params["encoder"])
        xc = _affine_center(buffers, batch)
        c = relu_code(xc, w, params["encoder_bias"])
        xc_hat = c @ w
        bd = buffers["bias_decay"] * torch.linalg.vector_norm(params["encoder_bias"])
        total, ld = _sae_losses(xc_hat, xc, c, buffers["l1_alpha"], bd)
        ld.pop("l_bias_decay")  # the reference's tied loss dict has no bias-decay key (:150-154)
        return total, (ld, {"c": c})


class FunctionalTiedCenteredSAE(DictSignature):
    """Tied SAE with a *learned* centering vector (reference sae_ensemble.py:162-228).
    Fused engine: ``FusedSAEEnsemble`` kind "tied_centered" (tied kernels on x - center)."""

    fused_kind = "tied_centered"

    @staticmethod
    def init(activation_size, n_dict_components, l1_alpha, center=None, device=None, dtype=None):
        dt = dtype or torch.float32
        params = {
            "center": center if center is not None else torch.zeros(activation_size, device=device, dtype=dt),
            "encoder": xavier((n_dict_components, activation_size), device, dtype),
            "encoder_bias": torch.zeros(n_dict_components, device=device, dtype=dt),
        }
        return params, {"l1_alpha": _scalar(l1_alpha, device, dtype)}

    @staticmethod
    def to_learned_dict(params, buffers):
        return TiedSAE(params["encoder"], params["encoder_bias"], centering=(params["center"], None, None),
                       norm_encoder=True)

    @staticmethod
    def loss(params, buffers, batch):
        w = unit_rows(params["encoder"])
        xc = batch - params["center"]
        c = relu_code(xc, w, params["encoder_bias"])
        total, ld = _sae_losses(c @ w, xc, c, buffers["l1_alpha"])
        return total, (ld, {"c": c})


# --------------------------------------------------------------------------- thresholding
def _smooth_threshold(c):
    return F.relu6(60.0 * (c - 0.9)) / 6.0 + F.relu(c - 1.0)


class FunctionalThresholdingSAE(DictSignature):
    """Smooth-threshold tied SAE with learned per-feature scale/gain (reference :230-288).

    fix B#10: the reference encodes with ``params["centering"]`` which ``init`` never
    creates; we add a zero-initialised learned ``centering`` vector so the model runs.
    Fused engine: ``FusedSAEEnsemble`` kind "threshold" (EPI_ENC_ACT / EPI_DC_ACT, act 2).
    """

    fused_kind = "threshold"

    @staticmethod
    def init(activation_size, n_dict_components, l1_alpha, device=None, dtype=None):
        dt = dtype or torch.float32
        params = {
            "encoder": xavier((n_dict_components, activation_size), device, dtype),
            "activation_scale": torch.ones(n_dict_components, device=device, dtype=dt),
            "activation_gain": torch.zeros(n_dict_components, device=device, dtype=dt),
            "centering": torch.zeros(activation_size, device=device, dtype=dt),
        }
        return params, {"l1_alpha": _scalar(l1_alpha, device, dtype)}

    @staticmethod
    def encode(params, batch, learned_dict):
        c = (batch - params["centering"]) @ learned_dict.transpose(-1, -2)
        a_sq = params["activation_scale"].pow(2)
        c = (c + params["activation_gain"]) / torch.clamp(a_sq, min=1e-8)
        return _smooth_threshold(c) * a_sq

    @staticmethod
    def loss(params, buffers, batch):
        w = unit_rows(params["encoder"])
        c = FunctionalThresholdingSAE.encode(params, batch, w)
        total, ld = _sae_losses(c @ w, batch, c, buffers["l1_alpha"])
        return total, (ld, {"c": c})

    @staticmethod
    def to_learned_dict(params, buffers):
        return ThresholdingSAE(params)


class ThresholdingSAE(LearnedDict):
    """Inference class of the thresholding SAE (reference sae_ensemble.py:290-303)."""

    def __init__(self, params):
        self.params = params
        self.n_feats, self.activation_size = params["encoder"].shape

    def get_learned_dict(self):
        return unit_rows(self.params["encoder"])

    def encode(self, batch):
        params = self.params
        if "centering" not in params:
            params = {**params, "centering": torch.zeros(self.activation_size, device=batch.device)}
        return FunctionalThresholdingSAE.encode(params, batch, self.get_learned_dict())

    def to_device(self, device):
        self.params = {k: v.to(device) for k, v in self.params.items()}


# --------------------------------------------------------------------------- masked
def _masked_buffers(n_dict_components, n_components_stack, l1_alpha, bias_decay, device, dtype):
    mask = torch.ones(n_components_stack, device=device, dtype=torch.bool)
    mask[:n_dict_components] = False
    return {
        "l1_alpha": _scalar(l1_alpha, device, dtype),
        "bias_decay": _scalar(bias_decay, device, dtype),
        "dict_size": torch.tensor(n_dict_components, device=device, dtype=torch.long),
        "coef_mask": mask,
    }


class FunctionalMaskedTiedSAE(DictSignature):
    """Tied SAEs of different sizes stacked by padding + code masking (reference :307-371)."""

    fused_kind = "tied"

    @staticmethod
    def init(activation_size, n_dict_components, n_components_stack, l1_alpha, bias_decay=0.0,
             device=None, dtype=None):
        params = {
            "encoder": xavier((n_components_stack, activation_size), device, dtype),
            "encoder_bias": torch.zeros(n_components_stack, device=device, dtype=dtype or torch.float32),
        }
        return params, _masked_buffers(n_dict_components, n_components_stack, l1_alpha, bias_decay, device, dtype)

    @staticmethod
    def to_learned_dict(params, buffers):
        n = int(buffers["dict_size"].item())
        return TiedSAE(params["encoder"][:n], params["encoder_bias"][:n], norm_encoder=True)

    @staticmethod
    def loss(params, buffers, batch):
        w = unit_rows(params["encoder"])
        c = relu_code(batch, w, params["encoder_bias"])
        c = c.masked_fill(buffers["coef_mask"], 0.0)
        total, ld = _sae_losses(c @ w, batch, c, buffers["l1_alpha"])
        return total, (ld, {"c": c})


class FunctionalMaskedSAE(DictSignature):
    """Untied masked SAE (reference sae_ensemble.py:375-442)."""

    fused_kind = "untied"

    @staticmethod
    def init(activation_size, n_dict_components, n_components_stack, l1_alpha, bias_decay=0.0,
             device=None, dtype=None):
        params = {
            "encoder": xavier((n_components_stack, activation_size), device, dtype),
            "encoder_bias": torch.zeros(n_components_stack, device=device, dtype=dtype or torch.float32),
            "decoder": xavier((n_components_stack, activation_size), device, dtype),
        }
        return params, _masked_buffers(n_dict_components, n_components_stack, l1_alpha, bias_decay, device, dtype)

    @staticmethod
    def to_learned_dict(params, buffers):
        n = int(buffers["dict_size"].item())
        return UntiedSAE(params["encoder"][:n], params["decoder"][:n], params["encoder_bias"][:n])

    @staticmethod
    def loss(params, buffers, batch):
        c = relu_code(batch, params["encoder"], params["encoder_bias"])
        c = c.masked_fill(buffers["coef_mask"], 0.0)
        total, ld = _sae_losses(c @ unit_rows(params["decoder"]), batch, c, buffers["l1_alpha"])
        return total, (ld, {"c": c})


# --------------------------------------------------------------------------- reverse
class FunctionalReverseSAE(DictSignature):
    """Tied SAE that subtracts the bias from active codes before decoding (reference :445-501).
    Fused engine: ``FusedSAEEnsemble`` kind "reverse" (EPI_ENC_ACT / EPI_DC_ACT, act 1)."""

    fused_kind = "reverse"

    @staticmethod
    def init(activation_size, n_dict_components, l1_alpha, bias_decay=0.0, device=None, dtype=None):
        params = {
            "encoder": xavier((n_dict_components, activation_size), device, dtype),
            "encoder_bias": torch.zeros(n_dict_components, device=device, dtype=dtype or torch.float32),
        }
        buffers = {"l1_alpha": _scalar(l1_alpha, device, dtype), "bias_decay": _scalar(bias_decay, device, dtype)}
        return params, buffers

    @staticmethod
    def to_learned_dict(params, buffers):
        return ReverseSAE(params["encoder"], params["encoder_bias"], norm_encoder=True)

    @staticmethod
    def loss(params, buffers, batch):
        w = unit_rows(params["encoder"])
        b = params["encoder_bias"]
        c = relu_code(batch, w, b)
        c = torch.where(c > 0.0, c - b, c)
        bd = buffers["bias_decay"] * torch.linalg.vector_norm(b)
        total, ld = _sae_losses(c @ w, batch, c, buffers["l1_alpha"], bd)
        return total, (ld, {"c": c})
