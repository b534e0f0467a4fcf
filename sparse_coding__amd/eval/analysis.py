"""Analysis experiments over trained dictionaries.

Reference: ``experiments/check_l0_tokens.py`` (do layer-0 features equal token
(un)embeddings?), ``experiments/investigate.py`` + ``standard_metrics.py:809-843``
(``run_mmcs_with_larger``: Hungarian-matched similarity of each dictionary with the
next larger one; effective number of neurons / entropy of converged vs unconverged
features), ``experiments/pca_perplexity.py`` (FVU vs perplexity of dictionaries,
PCA top-k / rotation baselines and added noise under reconstruction) and
``experiments/interp_moment_corrs.py`` (correlation of auto-interp scores with
activation moments).  All similarity maths are single GEMMs on the device.
"""

from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import metrics as M
from .interventions import perplexity_under_reconstruction


# ----------------------------------------------------------------------------- embeddings
def _unit(x: torch.Tensor) -> torch.Tensor:
    return x / x.norm(dim=-1, keepdim=True).clamp_min(1e-8)


def embed_unembed_similarity(lm, learned_dict) -> Tuple[float, float]:
    """Mean over atoms of the best cosine match to a token embedding / unembedding row."""
    emb = lm.model.get_input_embeddings().weight.detach().float()
    unemb = lm.model.get_output_embeddings().weight.detach().float()
    D = _unit(learned_dict.get_learned_dict().float().to(emb.device))
    e = float((D @ _unit(emb).T).max(dim=-1).values.mean())
    u = float((D @ _unit(unemb).T).max(dim=-1).values.mean())
    return e, u


# ----------------------------------------------------------------------------- convergence
def hungarian_max_cosine(small: torch.Tensor, large: torch.Tensor) -> np.ndarray:
    """Cosine similarity of each atom of ``small`` with its one-to-one match in ``large``."""
    from scipy.optimize import linear_sum_assignment

    sim = (_unit(small.float()) @ _unit(large.float().to(small.device)).T).cpu().numpy()
    r, c = linear_sum_assignment(1.0 - sim)
    out = np.zeros(small.shape[0])
    out[r] = sim[r, c]
    return out


def run_mmcs_with_larger(learned_dicts: Sequence[Sequence[torch.Tensor]], threshold: float = 0.9):
    """``learned_dicts[l1][size]`` -> (mean matched MMCS [L, S], % atoms above threshold [L, S],
    per-cell similarity arrays [L][S-1])."""
    L, S = len(learned_dicts), len(learned_dicts[0])
    av = np.zeros((L, S))
    above = np.zeros((L, S))
    full = [[None] * (S - 1) for _ in range(L)]
    for i in range(L):
        for j in range(S - 1):
            sims = hungarian_max_cosine(learned_dicts[i][j], learned_dicts[i][j + 1])
            av[i, j] = sims.mean()
            above[i, j] = (sims > threshold).mean() * 100
            full[i][j] = sims
    return av, above, full


def effective_number_of_neurons(features: torch.Tensor) -> torch.Tensor:
    p = features.abs() / features.abs().sum(dim=1, keepdim=True)
    return 1.0 / p.pow(2).sum(dim=1)


def feature_entropy(features: torch.Tensor) -> torch.Tensor:
    p = features.abs() / features.abs().sum(dim=1, keepdim=True)
    return -(p * torch.log(p + 1e-8)).sum(dim=1)


def converged_feature_stats(small: torch.Tensor, large: torch.Tensor, threshold: float = 0.9) -> Dict[str, float]:
    """ENN / entropy of atoms that reappear in the larger dictionary vs those that do not."""
    sims = torch.as_tensor(hungarian_max_cosine(small, large))
    conv = sims > threshold
    enn = effective_number_of_neurons(small.float().cpu())
    ent = feature_entropy(small.float().cpu())

    def m(x, mask):
        return float(x[mask].mean()) if mask.any() else float("nan")

    return {"frac_converged": float(conv.float().mean()), "enn_converged": m(enn, conv),
            "enn_unconverged": m(enn, ~conv), "entropy_converged": m(ent, conv), "entropy_unconverged": m(ent, ~conv)}


# ----------------------------------------------------------------------------- FVU vs perplexity
@torch.no_grad()
def fvu_vs_perplexity(lm, learned_dict_sets: Dict[str, List[Tuple[object, dict]]], sample: torch.Tensor,
                      tokens: torch.Tensor, location=(2, "residual"), batch: int = 16) -> Dict[str, List[Tuple[float, float]]]:
    """``{label: [(FVU, mean LM loss under reconstruction), ...]}`` (reference pca_perplexity.py)."""
    out = {}
    for label, items in learned_dict_sets.items():
        pts = []
        for ld, _ in items:
            ld.to_device(sample.device)
            fvu = float(M.fraction_variance_unexplained(ld, sample))
            losses = [float(perplexity_under_reconstruction(lm, ld, location, tokens[i:i + batch]))
                      for i in range(0, tokens.shape[0], batch)]
            pts.append((fvu, float(np.mean(losses))))
        out[label] = pts
    return out


def pca_baseline_sets(pca, d: int, step: int = 8) -> Dict[str, List[Tuple[object, dict]]]:
    """PCA (dynamic top-k) and PCA (static rotation) families for ``fvu_vs_perplexity``."""
    return {"PCA (dynamic)": [(pca.to_learned_dict(k), {"dict_size": d, "k": k}) for k in range(1, d // 2, step)],
            "PCA (static)": [(pca.to_rotation_dict(k), {"dict_size": d, "n": k}) for k in range(1, d // 2, step)]}


def added_noise_set(d: int, mags: Iterable[float], device="cpu") -> List[Tuple[object, dict]]:
    from ..models.learned_dict import AddedNoise

    return [(AddedNoise(float(m), d, device=device), {"dict_size": d, "noise": float(m)}) for m in mags]


# ----------------------------------------------------------------------------- interp-score correlations
def moment_score_correlations(learned_dict, activations: torch.Tensor, feature_idx: Sequence[int],
                              scores: Sequence[float], batch_size: int = 1000) -> Dict[str, float]:
    """Pearson correlation between auto-interp scores and each activation moment of the
    scored features (times active, mean, var, skew, kurtosis, 4th moment)."""
    moments = M.calc_moments_streaming(learned_dict, activations, batch_size)
    names = ["n_active", "mean", "var", "skew", "kurtosis", "l4_norm"]
    idx = torch.as_tensor(list(feature_idx), dtype=torch.long)
    s = torch.as_tensor(list(scores), dtype=torch.float64)
    out = {}
    for name, m in zip(names, moments):
        v = torch.as_tensor(m).detach().cpu().double()[idx]
        out[name] = float(torch.corrcoef(torch.stack([v, s]))[0, 1]) if len(s) > 1 else float("nan")
    return out
