"""Synthetic sparse-mixture activation generators.

Same generative models as reference ``sc_datasets/random_dataset.py:16-279``:

* ``RandomDatasetGenerator`` -- ``n`` unit-norm ground-truth features; feature
  ``i`` is active with probability ``decay**i * k / n`` (independent), active
  codes are ``U(0,1) * U(0,1)`` strengths; ``x = codes @ feats`` (:160-188).
* ``SparseMixDataset`` -- correlated activations: one multivariate-normal draw
  per batch passed through the normal CDF and the decay profile, rescaled so the
  mean activation probability is ``k / n``; every row gets at least one active
  feature; optional MVN noise (:76-157, :191-245).

Both are Python generators (``next(gen)`` / ``gen.send(batch_size)``) returning
``[batch, d]`` fp32 tensors on ``device``.  Unlike the reference they take an
explicit ``seed`` so runs are reproducible, and generation stays on the device
(``torch.Generator`` on the target device) instead of going through numpy.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Optional, Tuple, Union

import torch

Device = Union[str, torch.device]


def _gen(device, seed):
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    return g


def generate_rand_feats(feat_dim: int, num_feats: int, device: Device = "cpu", generator=None) -> torch.Tensor:
    """``num_feats`` random directions on the unit sphere in ``feat_dim`` dims."""
    f = torch.randn(num_feats, feat_dim, device=device, generator=generator)
    return f / f.norm(dim=1, keepdim=True)


def generate_corr_matrix(num_feats: int, device: Device = "cpu", generator=None) -> torch.Tensor:
    """Symmetric uniform random matrix shifted to be positive definite (reference :264-279)."""
    g64 = torch.rand(num_feats, num_feats, dtype=torch.float64, generator=generator,
                     device="cpu" if generator is None else generator.device)
    c = (g64 + g64.T) / 2
    min_eig = torch.linalg.eigvalsh(c).min()
    if min_eig < 0:
        c = c - 1.001 * min_eig * torch.eye(num_feats, dtype=torch.float64, device=c.device)
    return c.float().to(device)


def generate_rand_dataset(n_components, dataset_size, feature_probs, feats, device, generator=None
                          ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    thresh = torch.rand(dataset_size, n_components, device=device, generator=generator)
    values = torch.rand(dataset_size, n_components, device=device, generator=generator)
    codes = torch.where(thresh <= feature_probs, values, torch.zeros((), device=device))
    strengths = torch.rand(dataset_size, n_components, device=device, generator=generator)
    return feats, codes, (codes * strengths) @ feats


def generate_correlated_dataset(n_components, dataset_size, corr_matrix, feats, frac_nonzero, decay, device,
                                generator=None) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    chol = torch.linalg.cholesky(corr_matrix.double()).float()
    z = chol @ torch.randn(n_components, device=device, generator=generator)
    probs = torch.special.ndtr(z) * decay
    probs = probs * (frac_nonzero / probs.mean())
    thresh = torch.rand(dataset_size, n_components, device=device, generator=generator)
    values = torch.rand(dataset_size, n_components, device=device, generator=generator)
    codes = torch.where(thresh <= probs, values, torch.zeros((), device=device))
    empty = (codes != 0).sum(1) == 0
    if bool(empty.any()):
        rows = empty.nonzero()[:, 0]
        cols = torch.randint(0, n_components, (rows.numel(),), device=device, generator=generator)
        codes[rows, cols] = 1.0
    strengths = torch.rand(dataset_size, n_components, device=device, generator=generator)
    return feats, codes, (codes * strengths) @ feats


def generate_noise_dataset(dataset_size, noise_covariance, noise_magnitude_scale, device, generator=None):
    chol = torch.linalg.cholesky(noise_covariance.double()).float().to(device)
    z = torch.randn(dataset_size, noise_covariance.shape[0], device=device, generator=generator)
    return (z @ chol.T) * noise_magnitude_scale


class _GenBase:
    def __iter__(self):
        return self

    def __next__(self):
        return self.send(None)

    def throw(self, *args):
        raise StopIteration

    def close(self):
        pass


@dataclass
class RandomDatasetGenerator(_GenBase):
    activation_dim: int
    n_ground_truth_components: int
    batch_size: int
    feature_num_nonzero: int
    feature_prob_decay: float
    correlated: bool
    device: Device
    seed: int = 0
    # "hip": codes from the Philox kernel (ops/synth.py) and an MFMA GEMM, bf16 throughout (the
    # same distribution; a different random stream than the torch path)
    backend: str = "torch"

    frac_nonzero: float = field(init=False)
    decay: torch.Tensor = field(init=False)
    feats: torch.Tensor = field(init=False)
    corr_matrix: Optional[torch.Tensor] = field(init=False, default=None)
    component_probs: Optional[torch.Tensor] = field(init=False, default=None)

    def __post_init__(self):
        self.generator = _gen(self.device, self.seed)
        n = self.n_ground_truth_components
        self.frac_nonzero = self.feature_num_nonzero / n
        self.decay = self.feature_prob_decay ** torch.arange(n, device=self.device, dtype=torch.float32)
        if self.correlated:
            self.corr_matrix = generate_corr_matrix(n, device=self.device, generator=_gen("cpu", self.seed + 1))
        else:
            self.component_probs = self.decay * self.frac_nonzero
        self.feats = generate_rand_feats(self.activation_dim, n, device=self.device, generator=self.generator)
        self.t_type = torch.float32

    def send(self, ignored: Any = None) -> torch.Tensor:
        if self.backend == "hip":
            return self._send_hip()
        if self.correlated:
            _, _, data = generate_correlated_dataset(self.n_ground_truth_components, self.batch_size,
                                                     self.corr_matrix, self.feats, self.frac_nonzero, self.decay,
                                                     self.device, self.generator)
        else:
            _, _, data = generate_rand_dataset(self.n_ground_truth_components, self.batch_size,
                                               self.component_probs, self.feats, self.device, self.generator)
        return data.to(self.t_type)

    def _send_hip(self) -> torch.Tensor:
        from ..ops import synth

        if not hasattr(self, "_rows"):
            self._rows = 0
            self._feats_bf16 = self.feats.to(torch.bfloat16).contiguous()
        if self.correlated:  # one MVN draw per batch sets the per-feature probabilities
            chol = torch.linalg.cholesky(self.corr_matrix.double()).float()
            z = chol @ torch.randn(self.n_ground_truth_components, device=self.device, generator=self.generator)
            probs = torch.special.ndtr(z) * self.decay
            probs = probs * (self.frac_nonzero / probs.mean())
        else:
            probs = self.component_probs
        codes = synth.sparse_codes(probs, self.batch_size, self.seed, self._rows)
        self._rows += self.batch_size
        if self.correlated:  # every row gets at least one active feature (reference :236-240)
            empty = (codes != 0).sum(1) == 0
            if bool(empty.any()):
                rows = empty.nonzero()[:, 0]
                cols = torch.randint(0, self.n_ground_truth_components, (rows.numel(),), device=self.device,
                                     generator=self.generator)
                codes[rows, cols] = torch.rand(rows.numel(), device=self.device,
                                               generator=self.generator).to(codes.dtype)  # 1 x strength
        return synth.mix(codes, self._feats_bf16).to(self.t_type)


@dataclass
class SparseMixDataset(_GenBase):
    activation_dim: int
    n_sparse_components: int
    batch_size: int
    feature_num_nonzero: int
    feature_prob_decay: float
    noise_magnitude_scale: float
    device: Device
    sparse_component_dict: Optional[torch.Tensor] = None
    sparse_component_covariance: Optional[torch.Tensor] = None
    noise_covariance: Optional[torch.Tensor] = None
    t_type: Optional[torch.dtype] = None
    seed: int = 0

    def __post_init__(self):
        self.generator = _gen(self.device, self.seed)
        n = self.n_sparse_components
        self.frac_nonzero = self.feature_num_nonzero / n
        if self.sparse_component_dict is None:
            self.sparse_component_dict = generate_rand_feats(self.activation_dim, n, self.device, self.generator)
        if self.sparse_component_covariance is None:
            self.sparse_component_covariance = generate_corr_matrix(n, self.device, _gen("cpu", self.seed + 1))
        if self.noise_covariance is None:
            self.noise_covariance = torch.eye(self.activation_dim, device=self.device)
        self.sparse_component_probs = self.feature_prob_decay ** torch.arange(n, device=self.device,
                                                                                dtype=torch.float32)
        self.t_type = self.t_type or torch.float32

    def send(self, batch_size: Optional[int] = None) -> torch.Tensor:
        bs = self.batch_size if batch_size is None else batch_size
        _, _, sparse = generate_correlated_dataset(self.n_sparse_components, bs, self.sparse_component_covariance,
                                                   self.sparse_component_dict, self.frac_nonzero,
                                                   self.sparse_component_probs, self.device, self.generator)
        if self.noise_magnitude_scale:
            sparse = sparse + generate_noise_dataset(bs, self.noise_covariance, self.noise_magnitude_scale,
                                                     self.device, self.generator)
        return sparse.to(self.t_type)
