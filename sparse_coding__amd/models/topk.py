"""Top-k sparse coding (reference ``autoencoders/topk_encoder.py:8-62``).

``scores = x D_hat^T``; keep each row's k largest scores, ReLU; ``x_hat = code D_hat``;
loss = plain MSE (no L1).  k is a per-model buffer, which is why the reference needs
``no_stacking=True`` (``big_sweep_experiments.py:246-253``); the fused HIP path
(``ops.topk``) instead carries k per model in device memory and runs every model in
one launch.
"""

from __future__ import annotations

import torch
import torch.nn.functional as F

from .learned_dict import LearnedDict
from .signatures import DictSignature


def topk_codes(x, normed_dict, k, absolute: bool = False):
    """Dense [B, n] code with each row's top-k scores kept (ReLU unless ``absolute``)."""
    scores = x @ normed_dict.T
    key = scores.abs() if absolute else scores
    idx = torch.topk(key, int(k), dim=-1).indices
    code = torch.zeros_like(scores).scatter_(-1, idx, scores.gather(-1, idx))
    return code if absolute else F.relu(code)


class TopKEncoder(DictSignature):
    @staticmethod
    def init(d_activation, n_features, sparsity, dtype=torch.float32, device=None):
        params = {"dict": torch.randn(n_features, d_activation, dtype=dtype, device=device)}
        buffers = {"sparsity": torch.tensor(sparsity, dtype=torch.long, device=device)}
        return params, buffers

    @staticmethod
    def encode(b, sparsity, normed_dict):
        return topk_codes(b, normed_dict, int(sparsity))

    @staticmethod
    def loss(params, buffers, batch):
        D = params["dict"] / params["dict"].norm(dim=-1, keepdim=True)  # no clamp, as upstream
        code = TopKEncoder.encode(batch, buffers["sparsity"], D)
        loss = F.mse_loss(batch, code @ D)
        return loss, ({"loss": loss}, {"c": code})

    @staticmethod
    def to_learned_dict(params, buffers):
        D = params["dict"] / params["dict"].norm(dim=-1, keepdim=True)
        return TopKLearnedDict(D, int(buffers["sparsity"]))


class TopKLearnedDict(LearnedDict):
    def __init__(self, dict, sparsity):
        if not torch.is_tensor(dict):  # fix B#23: ICA passes numpy components
            dict = torch.as_tensor(dict, dtype=torch.float32)
        self.dict = dict
        self.sparsity = sparsity
        self.n_feats, self.activation_size = self.dict.shape

    def to_device(self, device):
        self.dict = self.dict.to(device)

    def encode(self, x):
        return topk_codes(x, self.dict, self.sparsity)

    def get_learned_dict(self):
        return self.dict
