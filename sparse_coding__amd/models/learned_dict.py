"""Inference-time dictionary objects (the ``LearnedDict`` API).

Behaviour follows reference ``autoencoders/learned_dict.py:13-274``: a learned
dictionary maps activations ``x [B, d]`` to codes ``c [B, n]`` (``encode``) and
back with ``x_hat = c @ D`` (``decode``), where ``D = get_learned_dict()`` is the
``[n, d]`` matrix of (usually unit-norm) atoms.  ``predict`` composes
``uncenter(decode(encode(center(x))))`` (reference ``learned_dict.py:42-47``).

Attribute names are kept identical to the reference (``encoder``,
``encoder_bias``, ``norm_encoder``, ``n_feats``, ``activation_size``,
``center_trans``/``center_rot``/``center_scale``) because they are part of the
pickled checkpoint format.  Deliberate fixes of reference
defects are marked "fix B#k" (SURVEY.md Appendix B).
"""

from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Optional

import torch


def _row_normalize(w: torch.Tensor, floor: float = 1e-8) -> torch.Tensor:
    return w / torch.clamp(w.norm(dim=-1), min=floor)[:, None]


class LearnedDict(ABC):
    """Abstract dictionary: subclasses provide ``get_learned_dict``, ``encode`` and ``to_device``."""

    n_feats: int
    activation_size: int

    @abstractmethod
    def get_learned_dict(self) -> torch.Tensor:
        """The ``[n_feats, activation_size]`` dictionary matrix."""

    @abstractmethod
    def encode(self, batch: torch.Tensor) -> torch.Tensor:
        """``[B, activation_size] -> [B, n_feats]`` codes."""

    @abstractmethod
    def to_device(self, device):
        """Move every tensor the dictionary owns to ``device``."""

    def decode(self, code: torch.Tensor) -> torch.Tensor:
        return code @ self.get_learned_dict()

    def center(self, batch: torch.Tensor) -> torch.Tensor:
        return batch

    def uncenter(self, batch: torch.Tensor) -> torch.Tensor:
        return batch

    def predict(self, batch: torch.Tensor) -> torch.Tensor:
        return self.uncenter(self.decode(self.encode(self.center(batch))))

    def n_dict_components(self) -> int:
        return self.get_learned_dict().shape[0]


class Identity(LearnedDict):
    """Codes are the activations themselves (reference learned_dict.py:53-65)."""

    def __init__(self, activation_size, device=None):
        self.n_feats = activation_size
        self.activation_size = activation_size
        self.device = device or "cpu"

    def get_learned_dict(self):
        return torch.eye(self.n_feats, device=self.device)

    def encode(self, batch):
        return batch

    def to_device(self, device):
        self.device = device


class IdentityReLU(LearnedDict):
    """``relu(x + bias)`` with the identity dictionary (reference learned_dict.py:68-85).

    fix B#22: the reference tests ``if bias:`` on a tensor; we test ``is not None``.
    """

    def __init__(self, activation_size, bias: Optional[torch.Tensor] = None):
        self.n_feats = activation_size
        self.activation_size = activation_size
        self.bias = bias if bias is not None else torch.zeros(activation_size)
        assert tuple(self.bias.shape) == (activation_size,)

    def get_learned_dict(self):
        return torch.eye(self.n_feats, device=self.bias.device)

    def encode(self, batch):
        return torch.clamp(batch + self.bias, min=0.0)

    def to_device(self, device):
        self.bias = self.bias.to(device)


class RandomDict(LearnedDict):
    """Gaussian random encoder used as a baseline (reference learned_dict.py:88-108)."""

    def __init__(self, activation_size, n_feats=None, generator=None):
        n_feats = n_feats or activation_size
        self.n_feats = n_feats
        self.activation_size = activation_size
        self.encoder = torch.randn(n_feats, activation_size, generator=generator)
        self.encoder_bias = torch.zeros(n_feats)

    def get_learned_dict(self):
        return self.encoder

    def encode(self, batch):
        return torch.clamp(batch @ self.encoder.T + self.encoder_bias, min=0.0)

    def to_device(self, device):
        self.encoder = self.encoder.to(device)
        self.encoder_bias = self.encoder_bias.to(device)


class UntiedSAE(LearnedDict):
    """``c = relu(W_e x + b)``, dictionary = row-normalised decoder (reference :111-131)."""

    def __init__(self, encoder, decoder, encoder_bias):
        self.encoder = encoder
        self.decoder = decoder
        self.encoder_bias = encoder_bias
        self.n_feats, self.activation_size = self.encoder.shape

    def get_learned_dict(self):
        return _row_normalize(self.decoder)

    def to_device(self, device):
        self.encoder = self.encoder.to(device)
        self.decoder = self.decoder.to(device)
        self.encoder_bias = self.encoder_bias.to(device)

    def encode(self, batch):
        return torch.clamp(batch @ self.encoder.T + self.encoder_bias, min=0.0)


class _CenteredTied(LearnedDict):
    """Shared implementation of the tied dictionaries with affine centering.

    ``center(x) = R (x - t) * s`` and ``uncenter(y) = R^T (y / s) + t``
    (reference learned_dict.py:166-170).  Missing centering attributes (old
    pickles) are back-filled with the identity transform (reference :156-164).
    """

    def __init__(self, encoder, encoder_bias, centering=(None, None, None), norm_encoder=False):
        self.encoder = encoder
        self.encoder_bias = encoder_bias
        self.norm_encoder = norm_encoder
        self.n_feats, self.activation_size = self.encoder.shape
        t, r, s = centering
        dev = encoder.device
        self.center_trans = t if t is not None else torch.zeros(self.activation_size, device=dev)
        self.center_rot = r if r is not None else torch.eye(self.activation_size, device=dev)
        self.center_scale = s if s is not None else torch.ones(self.activation_size, device=dev)

    def initialize_missing(self):
        dev = self.encoder.device
        if not hasattr(self, "center_trans"):
            self.center_trans = torch.zeros(self.activation_size, device=dev)
        if not hasattr(self, "center_rot"):
            self.center_rot = torch.eye(self.activation_size, device=dev)
        if not hasattr(self, "center_scale"):
            self.center_scale = torch.ones(self.activation_size, device=dev)

    def center(self, batch):
        self.initialize_missing()
        return ((batch - self.center_trans[None, :]) @ self.center_rot.T) * self.center_scale[None, :]

    def uncenter(self, batch):
        self.initialize_missing()
        return (batch / self.center_scale[None, :]) @ self.center_rot + self.center_trans[None, :]

    def get_learned_dict(self):
        return _row_normalize(self.encoder)

    def _enc_matrix(self):
        return _row_normalize(self.encoder) if self.norm_encoder else self.encoder

    def to_device(self, device):
        self.initialize_missing()
        self.encoder = self.encoder.to(device)
        self.encoder_bias = self.encoder_bias.to(device)
        self.center_trans = self.center_trans.to(device)
        self.center_rot = self.center_rot.to(device)
        self.center_scale = self.center_scale.to(device)

    def encode(self, batch):
        return torch.clamp(batch @ self._enc_matrix().T + self.encoder_bias, min=0.0)


class TiedSAE(_CenteredTied):
    """Tied-weights SAE (reference learned_dict.py:134-196)."""


class ReverseSAE(LearnedDict):
    """Tied SAE whose decoder removes the bias from active codes (reference :199-238).

    fix B#21: the reference mutates ``c`` in place inside ``decode``; we copy.
    The reference's ``einsum("dn,bn->bd")`` only type-checks for square
    dictionaries; we decode with the (row-normalised) dictionary as everywhere else.
    """

    def __init__(self, encoder, encoder_bias, norm_encoder=False):
        self.encoder = encoder
        self.encoder_bias = encoder_bias
        self.norm_encoder = norm_encoder
        self.n_feats, self.activation_size = self.encoder.shape

    def get_learned_dict(self):
        return _row_normalize(self.encoder)

    def _enc_matrix(self):
        return _row_normalize(self.encoder) if self.norm_encoder else self.encoder

    def to_device(self, device):
        self.encoder = self.encoder.to(device)
        self.encoder_bias = self.encoder_bias.to(device)

    def encode(self, batch):
        return torch.clamp(batch @ self._enc_matrix().T + self.encoder_bias, min=0.0)

    def decode(self, c):
        c = torch.where(c > 0.0, c - self.encoder_bias[None, :], c)
        return c @ self._enc_matrix()


class AddedNoise(LearnedDict):
    """``x + noise_mag * N(0, 1)`` baseline (reference learned_dict.py:241-255)."""

    def __init__(self, noise_mag, activation_size, device=None):
        self.noise_mag = noise_mag
        self.activation_size = activation_size
        self.n_feats = activation_size
        self.device = "cpu" if device is None else device

    def get_learned_dict(self):
        return torch.eye(self.activation_size, device=self.device)

    def to_device(self, device):
        self.device = device

    def encode(self, batch):
        return batch + torch.randn_like(batch) * self.noise_mag


class Rotation(LearnedDict):
    """A fixed linear map (e.g. the PCA basis) (reference learned_dict.py:258-274)."""

    def __init__(self, matrix, device=None):
        self.device = "cpu" if device is None else device
        self.matrix = matrix.to(self.device)
        self.activation_size = matrix.shape[1]
        self.n_feats = matrix.shape[0]

    def get_learned_dict(self):
        return self.matrix

    def to_device(self, device):
        self.matrix = self.matrix.to(device)
        self.device = device

    def encode(self, batch):
        return batch @ self.matrix.T
