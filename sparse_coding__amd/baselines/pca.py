"""Streaming PCA baseline (reference ``autoencoders/pca.py:6-126``).

The reference updates the covariance with ``einsum("bi,bj->bij")`` -- a [B, d, d]
temporary per batch.  Here the update is one SYRK-shaped GEMM (X_c^T X_c') per
batch, which on MI355X runs on the matrix cores via hipBLASLt and never
materialises [B, d, d].  Same Chan/Welford mean-covariance recurrence.
"""

from __future__ import annotations

import torch

from ..models.learned_dict import LearnedDict, Rotation
from ..models.topk import TopKLearnedDict


def calc_pca(activations, batch_size=512, device="cuda:0"):
    pca = BatchedPCA(activations.shape[1], device)
    for i in range(0, activations.shape[0], batch_size):
        pca.train_batch(activations[i:i + batch_size].to(device))
    return pca


def calc_mean(activations, batch_size=512, device="cuda:0"):
    mean = BatchedMean(activations.shape[1], device)
    for i in range(0, activations.shape[0], batch_size):
        mean.train_batch(activations[i:i + batch_size].to(device))
    return mean.get_mean()


class BatchedMean:
    def __init__(self, n_dims, device):
        self.n_dims = n_dims
        self.device = device
        self.mean = torch.zeros(n_dims, device=device, dtype=torch.float64)
        self.n_samples = 0

    def train_batch(self, activations):
        b = activations.shape[0]
        tot = self.n_samples + b
        self.mean = self.mean * (self.n_samples / tot) + activations.double().sum(0) / tot
        self.n_samples = tot

    def get_mean(self):
        return self.mean.float()


class BatchedPCA:
    def __init__(self, n_dims, device, dtype=torch.float64):
        self.n_dims = n_dims
        self.device = device
        self.cov = torch.zeros(n_dims, n_dims, device=device, dtype=dtype)
        self.mean = torch.zeros(n_dims, device=device, dtype=dtype)
        self.n_samples = 0

    def get_mean(self):
        return self.mean.float()

    def train_batch(self, activations):
        x = activations.to(self.cov.dtype)
        b = x.shape[0]
        tot = self.n_samples + b
        corrected = x - self.mean
        new_mean = self.mean + corrected.mean(0) * b / tot
        cov_update = corrected.T @ (x - new_mean) / b   # GEMM instead of a [B, d, d] einsum
        self.cov = self.cov * (self.n_samples / tot) + cov_update * (b / tot)
        self.mean = new_mean
        self.n_samples = tot

    def get_pca(self):
        vals, vecs = torch.linalg.eigh((self.cov + self.cov.T) / 2)
        return vals.float(), vecs.float()

    def get_centering_transform(self):
        vals, vecs = self.get_pca()
        scaling = 1.0 / torch.sqrt(torch.clamp(vals, min=1e-6))
        assert not torch.isnan(scaling).any(), "Scaling has NaNs"
        return self.get_mean(), vecs, scaling

    def get_dict(self):
        vals, vecs = self.get_pca()
        return vecs[:, torch.argsort(vals, descending=True)].T

    def to_learned_dict(self, sparsity):
        return PCAEncoder(self.get_dict(), sparsity)

    def to_topk_dict(self, sparsity):
        v = self.get_dict()
        return TopKLearnedDict(torch.cat([v, -v], dim=0), sparsity)

    def to_rotation_dict(self, n_components):
        return Rotation(self.get_dict()[:n_components])


class PCAEncoder(LearnedDict):
    """Keeps each row's top-k PCA scores by absolute value (reference pca.py:104-126)."""

    def __init__(self, pca_dict, sparsity):
        self.pca_dict = pca_dict / pca_dict.norm(dim=-1, keepdim=True)
        self.sparsity = sparsity
        self.n_feats, self.activation_size = self.pca_dict.shape

    def to_device(self, device):
        self.pca_dict = self.pca_dict.to(device)

    def encode(self, x):
        scores = x @ self.pca_dict.T
        idx = torch.topk(scores.abs(), self.sparsity, dim=-1).indices
        return torch.zeros_like(scores).scatter_(-1, idx, scores.gather(-1, idx))

    def get_learned_dict(self):
        return self.pca_dict
