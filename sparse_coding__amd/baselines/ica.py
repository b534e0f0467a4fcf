"""ICA and NMF baselines on CPU float64 via scikit-learn
(reference ``autoencoders/ica.py:15-53``, ``autoencoders/nmf.py:26-62``)."""

from __future__ import annotations

import time

import numpy as np
import torch

from ..models.learned_dict import LearnedDict
from ..models.topk import TopKLearnedDict


class ICAEncoder(LearnedDict):
    def __init__(self, activation_size, n_components: int = 0, seed: int = 0, max_iter: int = 200):
        from sklearn.decomposition import FastICA
        from sklearn.preprocessing import StandardScaler

        self.activation_size = activation_size
        self.n_feats = n_components or activation_size
        self.ica = FastICA(n_components=n_components or None, random_state=seed, max_iter=max_iter)
        self.scaler = StandardScaler()

    def to_device(self, device):
        for k in ("components", "offset", "scale"):
            if hasattr(self, k):
                setattr(self, k, getattr(self, k).to(device))

    def encode(self, x):
        """``((x - mu_s) / sigma_s - mu_ica) @ W^T`` -- sklearn's StandardScaler + FastICA
        transform as one affine map on the device (fp32)."""
        assert x.shape[1] == self.activation_size
        return ((x.float() - self.offset) / self.scale) @ self.components.T

    def train(self, dataset):
        """Fits on the CPU in float64, then keeps only tensors (components, offsets, scales),
        so a trained encoder runs on the GPU and loads with ``weights_only=True``."""
        assert dataset.shape[1] == self.activation_size
        xs = self.scaler.fit_transform(dataset.detach().cpu().numpy().astype(np.float64))
        t0 = time.time()
        out = self.ica.fit_transform(xs)
        self.fit_seconds = time.time() - t0
        mean_ica = self.ica.mean_ if getattr(self.ica, "mean_", None) is not None else 0.0
        scale = np.where(self.scaler.scale_ == 0, 1.0, self.scaler.scale_)
        self.components = torch.tensor(self.ica.components_, dtype=torch.float32)
        # (x - mu_s)/sigma - mu_ica == (x - (mu_s + sigma*mu_ica)) / sigma
        self.offset = torch.tensor(self.scaler.mean_ + scale * mean_ica, dtype=torch.float32)
        self.scale = torch.tensor(scale, dtype=torch.float32)
        self.n_feats = self.components.shape[0]
        self.ica = self.scaler = None
        return out

    def get_learned_dict(self):
        return self.components / self.components.norm(dim=-1, keepdim=True)

    def to_topk_dict(self, sparsity):
        comps = self.components
        return TopKLearnedDict(torch.cat([comps, -comps], dim=0), sparsity)


class NMFEncoder(LearnedDict):
    def __init__(self, activation_size, n_components=0, shift=0.0, seed: int = 0, max_iter: int = 200):
        from sklearn.decomposition import NMF

        self.activation_size = activation_size
        self.n_feats = n_components or activation_size
        self.nmf = NMF(n_components=n_components or None, random_state=seed, max_iter=max_iter)
        self.shift = shift

    def to_device(self, device):
        pass

    def encode(self, x):
        # fix B#21: does not mutate the caller's tensor
        xs = torch.clamp(x - self.shift, min=0.0)
        return torch.tensor(self.nmf.transform(xs.detach().cpu().numpy().astype(np.float64)), device=x.device,
                            dtype=torch.float32)

    def train(self, dataset):
        self.shift = min(float(self.shift), float(dataset.min()))
        data = (dataset - self.shift).detach().cpu().numpy().astype(np.float64)
        t0 = time.time()
        self.nmf.fit(data)
        self.fit_seconds = time.time() - t0

    def get_learned_dict(self):
        return torch.tensor(self.nmf.components_, dtype=torch.float32)

    def to_topk_dict(self, sparsity):
        return TopKLearnedDict(self.get_learned_dict(), sparsity)
