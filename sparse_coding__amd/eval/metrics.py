"""Dictionary quality metrics (reference ``standard_metrics.py``).

Every function takes a ``LearnedDict`` and activations ``[B, d]`` (or another
dictionary / ground-truth matrix) and returns tensors, so they run on CPU or
GPU unchanged.  Formulas follow SURVEY.md Appendix A:
``L0 = sum_j mean_b 1[c_bj != 0]`` on ``encode(center(x))`` and
``FVU = mean((x - predict(x))^2) / mean((x - mean_b x)^2)``.
Deliberate fixes of reference defects are tagged "fix B#k".
"""

from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np
import torch

from ..models.learned_dict import LearnedDict


# ------------------------------------------------------------------ sparsity / reconstruction
def mean_nonzero_activations(model: LearnedDict, batch: torch.Tensor) -> torch.Tensor:
    """Per-feature activation frequency (reference standard_metrics.py:303-306)."""
    c = model.encode(model.center(batch))
    return (c != 0).float().mean(dim=0)


def mean_l0(model: LearnedDict, batch: torch.Tensor) -> torch.Tensor:
    """Average number of active features per row (= sum of ``mean_nonzero_activations``)."""
    return mean_nonzero_activations(model, batch).sum()


def fraction_variance_unexplained(model: LearnedDict, batch: torch.Tensor) -> torch.Tensor:
    """Reference standard_metrics.py:308-312."""
    x_hat = model.predict(batch)
    resid = (batch - x_hat).pow(2).mean()
    total = (batch - batch.mean(dim=0)).pow(2).mean()
    return resid / total


def r_squared(model: LearnedDict, batch: torch.Tensor) -> torch.Tensor:
    return 1.0 - fraction_variance_unexplained(model, batch)


def fraction_variance_unexplained_top_activating(model: LearnedDict, batch: torch.Tensor, n_top: int = 2
                                                 ) -> Tuple[torch.Tensor, torch.Tensor]:
    """FVU using only the ``n_top`` most active features vs. the rest (reference :314-340).

    fix B#24: reconstructions are mapped back with ``uncenter`` (the reference applies ``center``).
    """
    c = model.encode(model.center(batch))
    order = torch.argsort(c.mean(dim=0), descending=True)
    top, rest = order[:n_top], order[n_top:]
    c_top = torch.zeros_like(c)
    c_top[:, top] = c[:, top]
    c_rest = torch.zeros_like(c)
    c_rest[:, rest] = c[:, rest]
    var = (batch - batch.mean(dim=0)).pow(2).mean()
    r_top = (batch - model.uncenter(model.decode(c_top))).pow(2).mean()
    r_rest = (batch - model.uncenter(model.decode(c_rest))).pow(2).mean()
    return r_top / var, r_rest / var


def batched_fvu_l0(model: LearnedDict, activations: torch.Tensor, batch_size: int = 8192
                   ) -> Tuple[float, float]:
    """Streaming FVU and L0 over a large activation set without materialising all codes."""
    n = activations.shape[0]
    mean = activations.float().mean(0)
    se = tot = 0.0
    l0 = 0.0
    for i in range(0, n, batch_size):
        x = activations[i:i + batch_size].float()
        c = model.encode(model.center(x))
        x_hat = model.uncenter(model.decode(c))
        se += float((x - x_hat).pow(2).sum())
        tot += float((x - mean).pow(2).sum())
        l0 += float((c != 0).sum())
    return se / tot, l0 / n


# ------------------------------------------------------------------ dictionary similarity
# Above this many similarity entries, GPU max-cosine reductions run on the fused
# EPI_ROWMAX kernel (bf16 MFMA, the [n1, n2] matrix never materialised; 16k x 16k fp32
# would be 1 GiB); below it the exact fp32 torch product is cheap enough.
ROWMAX_MIN_ENTRIES = 1 << 24


def max_cosine(rows: torch.Tensor, against: torch.Tensor, fused: bool | None = None) -> torch.Tensor:
    """max_j <rows_i, against_j> for every row (inputs already unit-norm)."""
    if fused is None:
        fused = rows.is_cuda and rows.shape[0] * against.shape[0] >= ROWMAX_MIN_ENTRIES
    if fused:
        from ..ops import gemm

        return gemm.rowmax_nt(rows.to(torch.bfloat16).contiguous(), against.to(torch.bfloat16).contiguous())
    return (rows @ against.T).max(dim=-1).values


def mcs_duplicates(ground: LearnedDict, model: LearnedDict) -> torch.Tensor:
    """Max cosine similarity of each ``model`` atom to the ``ground`` atoms (reference :268-272)."""
    return max_cosine(model.get_learned_dict(), ground.get_learned_dict())


def mmcs(model: LearnedDict, model2: LearnedDict) -> torch.Tensor:
    return mcs_duplicates(model, model2).mean()


def mcs_to_fixed(model: LearnedDict, truth: torch.Tensor) -> torch.Tensor:
    return max_cosine(model.get_learned_dict(), truth)


def mmcs_to_fixed(model: LearnedDict, truth: torch.Tensor) -> torch.Tensor:
    return mcs_to_fixed(model, truth).mean()


def mmcs_from_list(ld_list: Sequence[LearnedDict]) -> torch.Tensor:
    """Symmetric matrix of pairwise MMCS (reference :285-296)."""
    k = len(ld_list)
    out = torch.eye(k)
    for i in range(k):
        for j in range(i):
            out[i, j] = out[j, i] = float(mmcs(ld_list[i], ld_list[j]))
    return out


def representedness(features: torch.Tensor, model: LearnedDict) -> torch.Tensor:
    """For each ground-truth feature, max cosine similarity to any learned atom (reference :298-301)."""
    return (features @ model.get_learned_dict().T).max(dim=-1).values


def hungarian_mmcs(a: LearnedDict, b: LearnedDict) -> float:
    """Mean cosine similarity under the optimal one-to-one atom matching (reference :809-840)."""
    from scipy.optimize import linear_sum_assignment

    sim = (a.get_learned_dict() @ b.get_learned_dict().T).detach().float().cpu().numpy()
    r, c = linear_sum_assignment(-sim)
    return float(sim[r, c].mean())


# ------------------------------------------------------------------ dictionary geometry
def neurons_per_feature(model: LearnedDict) -> torch.Tensor:
    """Simpson-diversity count of neurons each atom uses (reference :345-350)."""
    D = model.get_learned_dict()
    p = D / D.abs().sum(dim=-1, keepdim=True)
    return (1.0 / p.pow(2).sum(dim=-1)).mean()


def capacity_per_feature(model: LearnedDict) -> torch.Tensor:
    """Capacity of Scherlis et al. 2022 (reference :354-360)."""
    D = model.get_learned_dict()
    sq = (D @ D.T).pow(2)
    return torch.diagonal(sq) / sq.sum(dim=-1)


# ------------------------------------------------------------------ activity statistics
def calc_feature_n_active(codes: torch.Tensor) -> torch.Tensor:
    return (codes != 0).sum(dim=0)


def batched_calc_feature_n_ever_active(learned_dict: LearnedDict, activations: torch.Tensor,
                                       batch_size: int = 1000, threshold: int = 10) -> int:
    """Number of features active more than ``threshold`` times (reference :444-452)."""
    counts = torch.zeros(learned_dict.n_feats, device=activations.device)
    for i in range(0, len(activations), batch_size):
        counts += calc_feature_n_active(learned_dict.encode(activations[i:i + batch_size]))
    return int((counts > threshold).sum())


def calc_feature_mean(codes):
    return codes.mean(dim=0)


def calc_feature_variance(codes):
    return codes.var(dim=0)


def calc_feature_skew(codes):
    var = codes.var(dim=0)
    return (codes ** 3).mean(dim=0) / torch.clamp(var ** 1.5, min=1e-8)


def calc_feature_kurtosis(codes):
    var = codes.var(dim=0)
    return (codes ** 4).mean(dim=0) / torch.clamp(var ** 2, min=1e-8)


def calc_moments_streaming(learned_dict: LearnedDict, activations: torch.Tensor, batch_size: int = 1000):
    """Streaming raw moments of every feature's activation (reference :454-509).

    fix B#25: a partial last batch is weighted by its true size and ``times_active`` counts
    samples (rows where the feature fired), not batches.
    Returns (times_active, mean, var, skew, kurtosis, m4).
    """
    nf = learned_dict.n_feats
    dev = activations.device
    times_active = torch.zeros(nf, device=dev)
    s1 = torch.zeros(nf, device=dev, dtype=torch.float64)
    s2 = torch.zeros_like(s1)
    s3 = torch.zeros_like(s1)
    s4 = torch.zeros_like(s1)
    n = 0
    for i in range(0, len(activations), batch_size):
        c = learned_dict.encode(activations[i:i + batch_size]).double()
        times_active += (c != 0).sum(0).float()
        s1 += c.sum(0)
        s2 += (c ** 2).sum(0)
        s3 += (c ** 3).sum(0)
        s4 += (c ** 4).sum(0)
        n += c.shape[0]
    mean, m2, m3, m4 = s1 / n, s2 / n, s3 / n, s4 / n
    var = m2 - mean ** 2
    skew = m3 / torch.clamp(var ** 1.5, min=1e-8)
    kurt = m4 / torch.clamp(var ** 2, min=1e-8)
    f = lambda t: t.float()
    return times_active, f(mean), f(var), f(skew), f(kurt), f(m4)


def ridge_regression_auroc(activations: torch.Tensor, labels: torch.Tensor, **kwargs) -> float:
    """Linear-probe AUROC (reference :252-258)."""
    from sklearn import metrics as skm
    from sklearn.linear_model import RidgeClassifier

    X, y = activations.detach().cpu().numpy(), labels.detach().cpu().numpy()
    clf = RidgeClassifier(**kwargs).fit(X, y)
    return float(skm.roc_auc_score(y, clf.predict(X)))


def cluster_vectors(learned_dict: LearnedDict, n_clusters: int = 100, top_clusters: int = 10,
                    seed: int = 0) -> List[List[int]]:
    """K-means over dictionary atoms; returns the feature indices of the largest clusters
    (reference standard_metrics.py:532-577, without the plotting)."""
    from sklearn.cluster import KMeans

    D = learned_dict.get_learned_dict().detach().float().cpu().numpy()
    km = KMeans(n_clusters=min(n_clusters, D.shape[0]), n_init=3, random_state=seed).fit(D)
    labels = km.labels_
    sizes = np.bincount(labels)
    order = np.argsort(-sizes)[:top_clusters]
    return [np.nonzero(labels == k)[0].tolist() for k in order]
