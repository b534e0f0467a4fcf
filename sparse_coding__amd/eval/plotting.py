"""Plots for sweep results (matplotlib, Agg backend; no display needed).

Reference: ``plotting/fvu_sparsity_plot.py:247-330`` (``plot_scores``),
``standard_metrics.py:362-530`` (``plot_capacities``, ``plot_capacity_scatter``,
``plot_hist``, ``plot_scatter``, ``plot_grid``), ``replicate_toy_models.py:356-397``
(``plot_mat``), ``plotting/plot_n_active*.py`` / ``num_dead_plot.py`` (active
features vs L1 per ratio) and ``plotting/plot_autointerp_violins.py`` (score
violins).  Image-returning helpers return a PIL image via ``canvas.buffer_rgba``
(``tostring_rgb``, which the reference uses, is gone from current matplotlib).

CLI: ``python -m sparse_coding__amd.eval.plotting fvu --dataset chunk.pt
--files "SAE=out/_9/learned_dicts.pt" "Fista=..." --out graphs/fvu``
"""

from __future__ import annotations

import argparse
import itertools
import os
from typing import Any, Dict, List, Optional, Sequence, Tuple

import matplotlib

matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402
from matplotlib.collections import LineCollection  # noqa: E402
from matplotlib.lines import Line2D  # noqa: E402

from . import metrics as M  # noqa: E402

COLORS = ["Purples", "Blues", "Greens", "Oranges", "Reds", "Greys"]
STYLES = ["x", "+", ".", "*", "o", "^"]


def default_settings(labels: Sequence[str], points: bool = True) -> Dict[str, dict]:
    combos = itertools.product(STYLES, COLORS)
    return {lab: {"style": s, "color": c, "points": points} for (s, c), lab in zip(combos, labels)}


def _to_image(fig):
    from PIL import Image

    fig.canvas.draw()
    buf = np.asarray(fig.canvas.buffer_rgba())[..., :3].copy()
    plt.close(fig)
    return Image.fromarray(buf, mode="RGB")


def plot_scores(scores, settings: Optional[dict], xlabel, ylabel, xrange, yrange, title, filename: Optional[str] = None,
                annotate: bool = False):
    """One series per label; points coloured by the optional third score (or lines)."""
    settings = settings or default_settings(list(scores))
    fig = plt.figure()
    ax = fig.add_subplot(111)
    handles, names = [], []
    norm = matplotlib.colors.Normalize(vmin=0, vmax=1)
    for label, pts in scores.items():
        cmap = matplotlib.colormaps[settings[label]["color"]]
        style = settings[label]["style"]
        pts = sorted(pts, key=lambda p: p[0])
        x = np.array([p[0] for p in pts])
        y = np.array([p[1] for p in pts])
        c = np.array([0.7 if p[2] is None else p[2] for p in pts], dtype=float)
        mc = float(c.mean()) if len(c) else 0.7
        if settings[label]["points"]:
            ax.scatter(x, y, c=c, cmap=cmap, norm=norm, marker=style, s=10)
            if annotate:
                for xi, yi in zip(x, y):
                    ax.text(xi, yi, f"{yi:.3g}", fontsize=8, ha="right", va="bottom")
            handles.append(Line2D([0], [0], color=cmap(mc), marker=style, linestyle="None", markersize=10))
        else:
            seg = np.concatenate([np.stack([x[:-1], y[:-1]], -1)[:, None], np.stack([x[1:], y[1:]], -1)[:, None]], 1)
            lc = LineCollection(seg, cmap=cmap, norm=norm, linestyle=style if style in ("-", "--", ":", "-.") else "-")
            lc.set_array(0.5 * (c[:-1] + c[1:]))
            lc.set_linewidth(2)
            ax.add_collection(lc)
            handles.append(Line2D([0], [0], color=cmap(mc), linewidth=2))
        names.append(label)
    ax.set_xlabel(xlabel)
    ax.set_ylabel(ylabel)
    ax.set_title(title)
    ax.set_xlim(*xrange)
    ax.set_ylim(*yrange)
    ax.legend(handles, names)
    if filename:
        os.makedirs(os.path.dirname(os.path.abspath(filename)), exist_ok=True)
        fig.savefig(f"{filename}.png")
    plt.close(fig)


def plot_mat(mat, l1_alphas, learned_dict_ratios, show=False, save_folder=None, save_name=None, title=None):
    """Heat map of an [n_l1, n_ratio] matrix (reference replicate_toy_models.py:356-397)."""
    assert mat.shape == (len(l1_alphas), len(learned_dict_ratios))
    fig = plt.figure()
    plt.imshow(np.asarray(mat).T, interpolation="nearest", cmap="viridis")
    plt.xticks(range(len(l1_alphas)), [f"{a:.2f}" for a in l1_alphas], rotation=90)
    plt.xlabel("l1_alpha")
    plt.yticks(range(len(learned_dict_ratios)), [str(r) for r in learned_dict_ratios])
    plt.ylabel("learned_dict_ratio")
    plt.colorbar()
    if title:
        plt.title(title)
    if save_folder:
        os.makedirs(save_folder, exist_ok=True)
        fig.savefig(os.path.join(save_folder, save_name))
    plt.close(fig)


def plot_grid(scores, first_tick_labels, second_tick_labels, first_label, second_label, **kwargs):
    fig = plt.figure()
    ax = fig.add_subplot(111)
    ax.imshow(scores, **kwargs)
    ax.set_xticks(np.arange(len(first_tick_labels)))
    ax.set_yticks(np.arange(len(second_tick_labels)))
    ax.set_xticklabels(first_tick_labels)
    ax.set_yticklabels(second_tick_labels)
    ax.set_xlabel(first_label)
    ax.set_ylabel(second_label)
    return _to_image(fig)


def plot_hist(scores, x_label, y_label, **kwargs):
    fig = plt.figure()
    ax = fig.add_subplot(111)
    ax.hist(np.asarray(torch.as_tensor(scores).cpu()), **kwargs)
    ax.set_xlabel(x_label)
    ax.set_ylabel(y_label)
    return _to_image(fig)


def plot_scatter(scores_x, scores_y, x_label, y_label, **kwargs):
    fig = plt.figure()
    ax = fig.add_subplot(111)
    ax.scatter(np.asarray(torch.as_tensor(scores_x).cpu()), np.asarray(torch.as_tensor(scores_y).cpu()), **kwargs)
    ax.set_xlabel(x_label)
    ax.set_ylabel(y_label)
    return _to_image(fig)


def plot_capacities(dicts, save_name: str = "capacities"):
    max_cap = dicts[0][0].get_learned_dict().shape[1]
    sums = [float(M.capacity_per_feature(ld).sum()) for ld, _ in dicts]
    l1 = [hp["l1_alpha"] for _, hp in dicts]
    fig = plt.figure()
    ax = fig.add_subplot(111)
    ax.scatter(l1, sums)
    ax.set_xlabel("L1 alpha")
    ax.set_ylabel("Sum of capacities")
    ax.set_xscale("log")
    ax.axhline(max_cap, color="red", linestyle="--")
    ax.set_ylim(0, max_cap * 1.1)
    ax.set_title(f"Sum of capacities vs L1 alpha - {save_name}")
    fig.savefig(save_name + ".png")
    plt.close(fig)


def plot_capacity_scatter(dicts, save_name: str = "capacity_scatter"):
    caps = []
    for i, (ld, _) in enumerate(dicts):
        c = M.capacity_per_feature(ld).cpu()
        fig = plt.figure()
        ax = fig.add_subplot(111)
        ax.scatter(range(len(c)), c)
        ax.set_xlabel("Learned feature")
        ax.set_ylabel("Capacity")
        ax.set_title(f"Capacity per feature - {save_name}")
        fig.savefig(f"{save_name}_{i}.png")
        plt.close(fig)
        caps.append(c)
    fig = plt.figure()
    ax = fig.add_subplot(111)
    ax.hist(torch.cat(caps).numpy(), bins=80)
    ax.set_xlabel("Capacity")
    ax.set_ylabel("Frequency")
    ax.set_title(f"Capacity histogram - {save_name}")
    fig.savefig(save_name + "_hist.png")
    plt.close(fig)


def plot_n_active(series: Dict[Any, List[Tuple[float, float]]], filename: str, title: str = "",
                  ylabel: str = "Fraction of features active"):
    """Active-feature fraction vs L1 per dictionary ratio (reference plot_n_active*.py)."""
    fig = plt.figure()
    ax = fig.add_subplot(111)
    for key, pts in series.items():
        pts = sorted(pts)
        ax.plot([p[0] for p in pts], [p[1] for p in pts], marker="o", label=str(key))
    ax.set_xscale("log")
    ax.set_xlabel("L1 alpha")
    ax.set_ylabel(ylabel)
    ax.set_title(title)
    ax.legend(title="ratio")
    fig.savefig(filename)
    plt.close(fig)


def plot_violins(scores: Dict[str, List[float]], filename: str, ylabel: str = "interpretability score",
                 xlabel: str = "Transform"):
    """Score distributions per transform (reference plot_autointerp_violins.py:60-131)."""
    names = [k for k in scores if len(scores[k]) > 1]  # a violin needs at least two samples
    fig = plt.figure(figsize=(max(6, len(names) * 0.9), 5))
    ax = fig.add_subplot(111)
    if names:
        ax.violinplot([scores[k] for k in names], showmeans=True)
    ax.set_xticks(range(1, len(names) + 1))
    ax.set_xticklabels(names, rotation=45, ha="right")
    ax.set_xlabel(xlabel)
    ax.set_ylabel(ylabel)
    fig.tight_layout()
    fig.savefig(filename)
    plt.close(fig)


# ----------------------------------------------------------------------------- CLI
def main(argv=None):
    from .scores import generate_scores, get_limits, load_sample

    p = argparse.ArgumentParser(description="FVU-vs-sparsity plot of learned-dict checkpoints")
    p.add_argument("kind", choices=["fvu"])
    p.add_argument("--dataset", required=True, help="activation chunk (.pt) to evaluate on")
    p.add_argument("--files", nargs="+", required=True, help="label=path/to/learned_dicts.pt")
    p.add_argument("--out", default="graphs/fvu_sparsity")
    p.add_argument("--x", default="sparsity")
    p.add_argument("--y", default="fvu")
    p.add_argument("--group_by", default="dict_size")
    p.add_argument("--n", type=int, default=50000)
    p.add_argument("--device", default="cuda:0" if torch.cuda.is_available() else "cpu")
    a = p.parse_args(argv)
    files = [tuple(f.split("=", 1)) if "=" in f else (os.path.basename(f), f) for f in a.files]
    sample = load_sample(a.dataset, n=a.n, device=a.device)
    scores = generate_scores(files, sample, a.x, a.y, group_by=a.group_by, label_format="{name} {val}")
    xr, yr = get_limits(scores)
    plot_scores(scores, None, a.x, a.y, (0, xr[1] * 1.05), (0, max(1.0, yr[1])), "FVU vs sparsity", a.out)
    for k, v in scores.items():
        print(k, [(round(x, 2), round(y, 4)) for x, y, _ in v])
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
