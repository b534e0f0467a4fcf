"""Score sets of learned dictionaries for plots: FVU / L0 / MMCS / top-FVU per dict,
grouped into labelled series, area under the FVU-sparsity curve, representedness,
ever-active fractions.

Reference: ``plotting/fvu_sparsity_plot.py:20-245`` (``score_dict``,
``area_under_fvu_sparsity_curve``, ``score_representedness``, ``generate_scores``,
``scores_derivative``, ``scores_logx/logy``), ``plotting/plot_n_active.py:35-118``
and ``standard_metrics.py:709-806`` (``calc_for_layer``/kurtosis jobs).  Checkpoints
are read with the safe loader (``utils.checkpoint.load_learned_dicts``); every
metric streams the evaluation sample in batches on the device.
"""

from __future__ import annotations

from collections import OrderedDict
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import metrics as M
from ..utils.checkpoint import load_learned_dicts

Series = Dict[str, List[Tuple[float, float, Optional[float]]]]


def _fvu_l0(ld, sample: torch.Tensor, batch: int = 16384):
    return M.batched_fvu_l0(ld, sample, batch)


def score_dict(score: str, hyperparams: dict, learned_dict, dataset: torch.Tensor, ground_truth=None) -> float:
    if score == "mcs":
        return float(M.mmcs_to_fixed(learned_dict, ground_truth))
    if score == "fvu":
        return float(M.fraction_variance_unexplained(learned_dict, dataset))
    if score == "sparsity":
        return float(M.mean_nonzero_activations(learned_dict, dataset).sum())
    if score == "l1":
        return float(hyperparams["l1_alpha"])
    if score == "neg_log_l1":
        return float(-np.log(hyperparams["l1_alpha"]))
    if score == "dict_size":
        return float(hyperparams["dict_size"])
    if score == "top_fvu":
        return float(M.fraction_variance_unexplained_top_activating(learned_dict, dataset)[0])
    if score == "rest_fvu":
        return float(M.fraction_variance_unexplained_top_activating(learned_dict, dataset)[1])
    raise ValueError(f"unknown score {score!r}")


def load_sample(dataset_file: Optional[str] = None, generator=None, n: int = 50000, device="cpu",
                seed: int = 0) -> torch.Tensor:
    """Evaluation sample: ``n`` random rows of a chunk file, or drawn from a generator."""
    if dataset_file is not None:
        data = torch.load(dataset_file, weights_only=True, map_location="cpu")
        g = torch.Generator().manual_seed(seed)
        idx = torch.randperm(data.shape[0], generator=g)[: min(n, data.shape[0])]
        return data[idx].to(device=device, dtype=torch.float32)
    rows, have = [], 0
    while have < n:
        rows.append(next(generator).to(device, torch.float32))
        have += rows[-1].shape[0]
    return torch.cat(rows)[:n]


def generate_scores(learned_dict_files: Sequence[Tuple[str, str]], dataset: torch.Tensor, x_score="sparsity",
                    y_score="fvu", c_score: Optional[str] = None, group_by="dict_size",
                    label_format="{name} {val:.2E}", ground_truth=None, device=None) -> Series:
    """``{series label: [(x, y, c), ...]}`` over every dictionary in the files."""
    device = device or dataset.device
    sets: "OrderedDict[str, list]" = OrderedDict()
    for label, path in learned_dict_files:
        for ld, hp in load_learned_dicts(path):
            val = hp.get(group_by, 0)
            try:
                name = label_format.format(name=label, val=val)
            except (ValueError, TypeError):
                name = f"{label} {val}"
            sets.setdefault(name, []).append((ld, hp))
    scores: Series = OrderedDict()
    for name, items in sets.items():
        pts = []
        for ld, hp in items:
            ld.to_device(device)
            with torch.no_grad():
                x = score_dict(x_score, hp, ld, dataset, ground_truth)
                y = score_dict(y_score, hp, ld, dataset, ground_truth)
                c = score_dict(c_score, hp, ld, dataset, ground_truth) if c_score else None
            pts.append((x, y, c))
        scores[name] = pts
    return scores


def area_under_fvu_sparsity_curve(learned_dict_files, dataset: torch.Tensor) -> List[Tuple[int, float]]:
    """Per dict size: trapezoid area of L0 vs clipped FVU, anchored at (1, 0) and (0, d)."""
    d = dataset.shape[1]
    series: Dict[int, List[Tuple[float, float]]] = {}
    for _, path in learned_dict_files:
        for ld, hp in load_learned_dicts(path):
            ld.to_device(dataset.device)
            fvu, l0 = _fvu_l0(ld, dataset)
            series.setdefault(hp["dict_size"], [(1.0, 0.0), (0.0, float(d))]).append(
                (float(np.clip(fvu, 0, 1)), float(l0)))
    out = []
    for size, pts in series.items():
        pts = sorted(pts, key=lambda p: p[0])
        x, y = zip(*pts)
        out.append((size, float(np.trapezoid(y, x) if hasattr(np, "trapezoid") else np.trapz(y, x))))
    return out


def score_representedness(learned_dict_files, ground_truth: torch.Tensor) -> Dict[Tuple, float]:
    scores: Dict[Tuple, List[float]] = {}
    for _, path in learned_dict_files:
        for ld, hp in load_learned_dicts(path):
            ld.to_device(ground_truth.device)
            key = tuple(sorted(hp.items()))
            scores.setdefault(key, []).append(float(M.representedness(ground_truth, ld).mean()))
    return {k: float(np.mean(v)) for k, v in scores.items()}


def scores_derivative(scores: Series) -> Series:
    """d(y)/d(x) between consecutive points of each series (sorted by x)."""
    out: Series = OrderedDict()
    for name, pts in scores.items():
        pts = sorted(pts, key=lambda p: p[0])
        out[name] = [((a[0] + b[0]) / 2, (b[1] - a[1]) / (b[0] - a[0] + 1e-12), a[2]) for a, b in zip(pts, pts[1:])]
    return out


def scores_logx(scores: Series) -> Series:
    return OrderedDict((k, [(float(np.log(x)), y, c) for x, y, c in v]) for k, v in scores.items())


def scores_logy(scores: Series) -> Series:
    return OrderedDict((k, [(x, float(np.log(y)), c) for x, y, c in v]) for k, v in scores.items())


def get_limits(scores: Series) -> Tuple[Tuple[float, float], Tuple[float, float]]:
    xs = [p[0] for v in scores.values() for p in v]
    ys = [p[1] for v in scores.values() for p in v]
    return (min(xs), max(xs)), (min(ys), max(ys))


@torch.no_grad()
def n_active_table(dicts: Iterable[Tuple[object, dict]], activations: torch.Tensor, threshold: int = 10,
                   batch_size: int = 50000, with_kurtosis: bool = False) -> List[dict]:
    """Per dictionary: fraction of features firing more than ``threshold`` times on
    ``activations`` (reference calc_for_layer) and optionally mean kurtosis over all / active
    features (calc_kurtosis_for_layer)."""
    rows = []
    for ld, hp in dicts:
        ld.to_device(activations.device)
        n_feats = ld.get_learned_dict().shape[0]
        counts = torch.zeros(n_feats, device=activations.device)
        kurt = torch.zeros(n_feats, device=activations.device)
        nb = 0
        for i in range(0, activations.shape[0], batch_size):
            c = ld.encode(activations[i:i + batch_size].float())
            counts += (c != 0).sum(0)
            if with_kurtosis:
                kurt += M.calc_feature_kurtosis(c)
            nb += 1
        active = counts > threshold
        rec = dict(hp)
        rec.update(n_active=int(active.sum()), frac_active=float(active.float().mean()))
        if with_kurtosis:
            kurt /= max(nb, 1)
            rec.update(kurtosis_all=float(kurt.mean()),
                       kurtosis_active=float(kurt[active].mean()) if active.any() else float("nan"))
        rows.append(rec)
    return rows
