"""Sweep-result, FVU/sparsity-area, KL-divergence, bottleneck and auto-interp-trend plots.

Reference scripts (hard-coded paths there; functions over in-memory scores here):
- ``plotting/plot_sweep_results.py:29-412``: grouping sweep output folders by layer /
  location / dictionary ratio / tied-ness and plotting FVU against sparsity per group;
- ``plotting/fvu_sparsity_plot*.py``: FVU (or top-activation FVU) vs L0 curves with the
  area under them (``eval/scores.py`` computes the areas);
- ``plotting/plot_kl_div.py``: sparsity vs KL divergence of the model's output under
  reconstruction;
- ``plotting/bottleneck_plot.py``: KL divergence vs number of uncorrupted features;
- ``plotting/plot_autointerp_across_{chunks,size}.py``: auto-interpretation score means
  with 95% confidence intervals per layer, one series per transform (training length or
  dictionary size).

Output folders of the sweeps are named ``{tied|untied}_{loc}_l{layer}_r{ratio}[...]`` with
chunk checkpoints ``_{chunk}/learned_dicts.pt`` inside (``train/sweep.py``).
"""

from __future__ import annotations

import os
import re
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import matplotlib

matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402
import numpy as np  # noqa: E402

Series = Dict[str, List[Tuple[float, float]]]

_RUN_RE = re.compile(r"(?P<tied>untied|tied)?.*?_(?P<loc>residual|resid|mlpout|mlp|attn)_l(?P<layer>\d+)_r(?P<ratio>[\d.]+)")


def parse_run_name(name: str) -> Optional[dict]:
    """``tied_mlp_l3_r4`` -> {tied: True, loc: "mlp", layer: 3, ratio: 4.0, long: False}
    (reference plot_sweep_results.py:35-60 filters by the same substrings)."""
    m = _RUN_RE.search(os.path.basename(name.rstrip("/")))
    if not m:
        return None
    loc = m.group("loc")
    return {"tied": m.group("tied") != "untied" and m.group("tied") is not None, "loc": "residual" if loc == "resid" else loc,
            "layer": int(m.group("layer")), "ratio": float(m.group("ratio").rstrip(".")), "long": "long" in name}


def find_runs(root: str, chunk: Optional[int] = None, **filters) -> List[Tuple[dict, str]]:
    """Sweep output folders under ``root`` with their ``learned_dicts.pt`` (the given chunk, or the
    last one present), filtered on parsed fields (``loc="mlp", tied=True, layer=3``)."""
    out = []
    for name in sorted(os.listdir(root)):
        meta = parse_run_name(name)
        if meta is None or any(meta.get(k) != v for k, v in filters.items()):
            continue
        folder = os.path.join(root, name)
        chunks = sorted((int(c[1:]) for c in os.listdir(folder) if re.fullmatch(r"_\d+", c)
                         and os.path.exists(os.path.join(folder, c, "learned_dicts.pt"))))
        if not chunks:
            continue
        c = chunk if chunk is not None and chunk in chunks else chunks[-1]
        out.append((dict(meta, chunk=c), os.path.join(folder, f"_{c}", "learned_dicts.pt")))
    out.sort(key=lambda t: (t[0]["layer"], t[0]["loc"], t[0]["ratio"]))
    return out


def sweep_series(runs: Sequence[Tuple[dict, str]], sample, x_score: str = "sparsity", y_score: str = "fvu",
                 label_format: str = "{loc} l{layer} r{ratio:g}{tied_s}") -> Series:
    """One (x, y) series per run folder over its L1 sweep, scored on ``sample`` (reference
    plot_sweep_results.py:112-190)."""
    from ..utils.checkpoint import load_learned_dicts
    from .scores import score_dict

    series: Series = {}
    for meta, path in runs:
        label = label_format.format(tied_s=" tied" if meta["tied"] else "", **meta)
        pts = []
        for ld, hp in load_learned_dicts(path):
            ld.to_device(sample.device)
            pts.append((score_dict(x_score, hp, ld, sample), score_dict(y_score, hp, ld, sample)))
        series[label] = sorted(pts)
    return series


def plot_sweep_grid(grid: Dict[Tuple[str, str], Series], filename: str, xlabel: str = "mean L0",
                    ylabel: str = "FVU", logx: bool = True, title: str = "") -> str:
    """Grid of panels keyed by (row, column) -- e.g. (layer, location) -- each with one line per
    series (dictionary ratio / tied-ness), as the reference's per-group sweep figures."""
    rows = sorted({r for r, _ in grid}, key=str)
    cols = sorted({c for _, c in grid}, key=str)
    fig, axes = plt.subplots(len(rows), len(cols), figsize=(4 * len(cols), 3.2 * len(rows)), squeeze=False)
    cmap = plt.get_cmap("viridis")
    for (r, c), series in grid.items():
        ax = axes[rows.index(r)][cols.index(c)]
        for k, (label, pts) in enumerate(series.items()):
            if not pts:
                continue
            xs, ys = zip(*pts)
            ax.plot(xs, ys, marker="o", ms=3, color=cmap(k / max(1, len(series) - 1)), label=label)
        if logx:
            ax.set_xscale("log")
        ax.set_title(f"{r} / {c}", fontsize=9)
        ax.set_xlabel(xlabel)
        ax.set_ylabel(ylabel)
        ax.grid(True, alpha=0.3, linestyle="dashed")
        ax.legend(fontsize=6)
    if title:
        fig.suptitle(title)
    fig.tight_layout()
    fig.savefig(filename, dpi=120)
    plt.close(fig)
    return filename


def plot_fvu_sparsity_area(series: Series, filename: str, activation_width: int, ylabel: str = "FVU",
                           title: str = "") -> Dict[str, float]:
    """FVU vs L0 curves with the area under each, as reference fvu_sparsity_plot.py:40-78:
    the points (fvu clipped to [0, 1], sparsity) are closed with (fvu 1, L0 0) and
    (fvu 0, L0 = width), sorted by fvu, and the area is the integral of L0 over fvu (divided
    by the width here).  ``ylabel="top-activation FVU"`` for the top_fvu variant."""
    fig, ax = plt.subplots(figsize=(6, 4))
    areas = {}
    cmap = plt.get_cmap("tab10")
    for k, (label, pts) in enumerate(series.items()):
        closed = sorted([(1.0, 0.0), (0.0, float(activation_width)),
                         *[(float(np.clip(y, 0, 1)), float(x)) for x, y in pts]])
        fv, sp = zip(*closed)
        area = float(np.trapezoid(sp, fv) / activation_width)
        areas[label] = area
        order = np.argsort(sp)
        xs, ys = np.asarray(sp)[order], np.asarray(fv)[order]
        ax.plot(xs, ys, color=cmap(k % 10), label=f"{label} (area {area:.3f})")
        ax.fill_between(xs, ys, alpha=0.12, color=cmap(k % 10))
    ax.set_xscale("symlog", linthresh=1.0)
    ax.set_xlabel("mean L0")
    ax.set_ylabel(ylabel)
    ax.set_ylim(0, 1.05)
    ax.legend(fontsize=7)
    if title:
        ax.set_title(title)
    fig.tight_layout()
    fig.savefig(filename, dpi=120)
    plt.close(fig)
    return areas


def plot_kl_div(scores: Dict[str, Sequence[Tuple[float, float]]], filename: str) -> str:
    """Sparsity against KL divergence of the model's next-token distribution under
    reconstruction, one line per dictionary family (reference plot_kl_div.py)."""
    fig, ax = plt.subplots()
    for label, pts in scores.items():
        kl, sp = zip(*pts)
        ax.plot(kl, sp, marker=".", label=label)
    ax.set_xlabel("KL divergence")
    ax.set_ylabel("sparsity (mean L0)")
    ax.legend()
    fig.savefig(filename, dpi=120)
    plt.close(fig)
    return filename


def plot_bottleneck(scores: Dict[str, Sequence[Tuple[Sequence[int], float, float]]], filename: str,
                    layer: Optional[int] = None, xmax: Optional[int] = None) -> str:
    """Precision-complexity trade-off: KL divergence from the base model against the number of
    uncorrupted features, per dictionary (entries are (feature graph, divergence, corruption);
    reference bottleneck_plot.py:12-79)."""
    fig, ax = plt.subplots()
    ax.grid(True, alpha=0.5, linestyle="dashed")
    ax.set_axisbelow(True)
    for label, entries in scores.items():
        entries = sorted(entries, key=lambda e: len(e[0]))
        ax.plot([len(g) for g, _, _ in entries], [dv for _, dv, _ in entries],
                linestyle="dotted" if label.lower().startswith("pca") else "dashed", label=label)
    ax.set_xlabel("no. uncorrupted features")
    ax.set_ylabel("KL divergence from base")
    ax.set_title("precision-complexity trade-off" + (f" - layer {layer}" if layer is not None else ""))
    if xmax:
        ax.set_xlim(0, xmax)
    ax.legend(loc="upper right", framealpha=1)
    fig.savefig(filename, dpi=120)
    plt.close(fig)
    return filename


def mean_ci(scores: Iterable[float]) -> Tuple[float, float]:
    """Mean and 95% normal-approximation half-width (1.96 s / sqrt(n))."""
    a = np.asarray(list(scores), dtype=np.float64)
    if a.size == 0:
        return float("nan"), float("nan")
    ci = 1.96 * a.std(ddof=1) / np.sqrt(a.size) if a.size > 1 else 0.0
    return float(a.mean()), float(ci)


def plot_autointerp_trend(per_group: Sequence[Dict[str, Sequence[float]]], transforms: Sequence[str],
                          group_labels: Sequence[str], filename: str, xlabel: str = "layer",
                          ylabel: str = "mean auto-interp score", ylim: Optional[Tuple[float, float]] = (0, 0.34)) -> str:
    """Grouped error bars: for every group (layer) the mean and 95% CI of each transform's
    scores (reference plot_autointerp_across_chunks.py / _across_size.py: transforms are
    training lengths ``..._nc{n}`` or dictionary sizes ``..._r{ratio}``)."""
    fig, ax = plt.subplots(figsize=(7, 4))
    width = 0.8 / max(1, len(transforms))
    cmap = plt.get_cmap("tab10")
    for t, name in enumerate(transforms):
        xs, ms, cs = [], [], []
        for gi, scores in enumerate(per_group):
            if name in scores and len(scores[name]):
                m, ci = mean_ci(scores[name])
                xs.append(gi + 1 + (t - (len(transforms) - 1) / 2) * width)
                ms.append(m)
                cs.append(ci)
        if xs:
            ax.errorbar(xs, ms, yerr=cs, fmt="o", capsize=3, color=cmap(t % 10), label=name)
    ax.set_xticks(range(1, len(group_labels) + 1), list(group_labels))
    ax.set_xlabel(xlabel)
    ax.set_ylabel(ylabel)
    if ylim:
        ax.set_ylim(*ylim)
    ax.grid(axis="y", color="grey", linewidth=0.5, alpha=0.3)
    ax.legend(fontsize=7)
    fig.tight_layout()
    fig.savefig(filename, dpi=120)
    plt.close(fig)
    return filename
