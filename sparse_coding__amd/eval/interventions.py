"""Model-level evaluation of dictionaries: reconstruction interventions, perplexity
under reconstruction, feature ablation graphs, probe AUROC.

Reference: ``standard_metrics.py:36-250`` (``run_with_model_intervention``,
``ablate_feature_intervention[_non_positional]``, ``cache_all_activations``,
``build_ablation_graph[_non_positional]``, ``perplexity_under_reconstruction``,
``logistic_regression_auroc``) and ``:619-706`` (``calculate_perplexity``).
Runs on ``interp.hooked.HookedLM``.  Differences: the ablation graph encodes each
location once per ablation with all target features gathered in one indexing op
(the reference loops per target in Python), and ``calculate_perplexity`` takes
token batches (no HF-datasets download; B#22-style hard-coded devices removed).
"""

from __future__ import annotations

from itertools import product
from typing import Dict, Iterable, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from ..interp.hooked import HookedLM, tensor_name

Location = Tuple[int, str]
FeatureIdx = Tuple[int, int]   # (position, feature)
Feature = Tuple[Location, FeatureIdx]


def get_model_tensor_name(location: Location) -> str:
    if location[1] not in ("residual", "mlp"):
        raise ValueError(f"Location '{location[1]}' not supported")
    return tensor_name(location[0], location[1])


def _predict_bsd(model, t: torch.Tensor) -> torch.Tensor:
    B, L, C = t.shape
    return model.predict(t.reshape(B * L, C).to(torch.float32)).reshape(B, L, C).to(t.dtype)


def run_with_model_intervention(transformer: HookedLM, model, tensor_name_: str, tokens, other_hooks=(), **kwargs):
    """Forward with the hook tensor replaced by the dictionary's reconstruction."""
    return transformer.run_with_hooks(tokens, fwd_hooks=list(other_hooks) + [(tensor_name_, lambda t, hook=None:
                                                                             _predict_bsd(model, t))], **kwargs)


def perplexity_under_reconstruction(transformer: HookedLM, model, location: Location, tokens, **kwargs):
    """LM loss with the activation at ``location`` replaced by ``model.predict``."""
    return transformer.run_with_hooks(tokens, fwd_hooks=[(get_model_tensor_name(location),
                                                          lambda t, hook=None: _predict_bsd(model, t))],
                                      return_type="loss", **kwargs)


def ablate_feature_intervention(model, location: Location, feature: FeatureIdx):
    """Subtract feature ``feature[1]``'s contribution at position ``feature[0]``."""
    pos, idx = feature

    def go(t, hook=None):
        c = model.encode(t[:, pos, :].float())
        d = model.get_learned_dict()
        t[:, pos, :] -= (c[:, idx:idx + 1] * d[idx][None, :]).to(t.dtype)
        return t

    return go


def ablate_feature_intervention_non_positional(model, location: Location, feature_idx: int):
    def go(t, hook=None):
        B, L, C = t.shape
        c = model.encode(t.reshape(B * L, C).float())
        d = model.get_learned_dict()
        t -= (c[:, feature_idx:feature_idx + 1] * d[feature_idx][None, :]).reshape(B, L, C).to(t.dtype)
        return t

    return go


def cache_all_activations(transformer: HookedLM, models: Dict[Location, object], tokens, fwd_hooks=()):
    """Dictionary codes ``[B, S, n]`` at every location in ``models``, one forward."""
    names = {loc: get_model_tensor_name(loc) for loc in models}
    _, cache = transformer.run_with_cache(tokens, names_filter=list(names.values()), fwd_hooks=fwd_hooks,
                                          return_type=None)
    out = {}
    for loc, m in models.items():
        t = cache[names[loc]]
        B, L, C = t.shape
        out[loc] = m.encode(t.reshape(B * L, C).float()).reshape(B, L, -1)
    return out


def _graph(transformer, models, tokens, features_to_ablate, target_features, make_hook, select):
    all_features = [(loc, f) for loc, fs in {**features_to_ablate, **target_features}.items() for f in fs]
    base = cache_all_activations(transformer, models, tokens)
    by_loc: Dict[Location, List] = {}
    for loc, f in all_features:
        by_loc.setdefault(loc, []).append(f)
    graph = {}
    for loc, m in models.items():
        for feat in features_to_ablate.get(loc, []):
            abl = cache_all_activations(transformer, models, tokens,
                                        fwd_hooks=[(get_model_tensor_name(loc), make_hook(m, loc, feat))])
            for loc2, feats in by_loc.items():
                diffs = select(base[loc2], feats) - select(abl[loc2], feats)  # [B(,S), n_targets]
                norms = diffs.norm(dim=-2) if diffs.dim() == 2 else diffs.norm(dim=-2).mean(0)
                for f2, v in zip(feats, norms.tolist()):
                    if loc2 == loc and f2 == feat:
                        continue
                    graph[(loc, feat), (loc2, f2)] = v
    return graph


def build_ablation_graph(transformer: HookedLM, models: Dict[Location, object], tokens,
                         features_to_ablate: Optional[Dict[Location, List[FeatureIdx]]] = None,
                         target_features: Optional[Dict[Location, List[FeatureIdx]]] = None):
    """Edge weight = mean over sentences of |Δ activation| of a target (position, feature)
    when a source (position, feature) is ablated (reference standard_metrics.py:115-158)."""
    B, L = tokens.shape
    if not features_to_ablate:
        features_to_ablate = {loc: list(product(range(L), range(m.get_learned_dict().shape[0])))
                              for loc, m in models.items()}

    def select(codes, feats):
        pos = torch.tensor([p for p, _ in feats], device=codes.device)
        idx = torch.tensor([i for _, i in feats], device=codes.device)
        return codes[:, pos, idx]                    # [B, n_targets]

    def wrap(m, loc, feat):
        return ablate_feature_intervention(m, loc, feat)

    return _graph(transformer, models, tokens, features_to_ablate, target_features or {}, wrap, select)


def build_ablation_graph_non_positional(transformer: HookedLM, models: Dict[Location, object], tokens,
                                        features_to_ablate: Optional[Dict[Location, List[int]]] = None,
                                        target_features: Optional[Dict[Location, List[int]]] = None):
    """Reference standard_metrics.py:177-219: norm over positions, mean over sentences."""
    if not features_to_ablate:
        features_to_ablate = {loc: list(range(m.get_learned_dict().shape[0])) for loc, m in models.items()}

    def select(codes, feats):
        return codes[:, :, torch.tensor(feats, device=codes.device)]  # [B, S, n_targets]

    return _graph(transformer, models, tokens, features_to_ablate, target_features or {},
                  ablate_feature_intervention_non_positional, select)


@torch.no_grad()
def calculate_perplexity(transformer: HookedLM, autoencoders, layer: int, setting: str,
                         token_batches: Iterable[torch.Tensor]) -> Tuple[float, List[float]]:
    """Original perplexity and perplexity with each dictionary's reconstruction spliced in
    (reference standard_metrics.py:619-706)."""
    if isinstance(autoencoders, tuple):
        autoencoders = [autoencoders]
    assert setting in ("residual", "mlp"), "setting must be either 'residual' or 'mlp'"
    batches = [b for b in token_batches]
    base = torch.stack([transformer(b, return_type="loss") for b in batches]).mean()
    out = []
    for ae, _ in autoencoders:
        ae.to_device(transformer.device)
        losses = [perplexity_under_reconstruction(transformer, ae, (layer, setting), b) for b in batches]
        out.append(float(torch.exp(torch.stack(losses).mean())))
    return float(torch.exp(base)), out


def logistic_regression_auroc(activations: torch.Tensor, labels: torch.Tensor, **kwargs) -> float:
    from sklearn.linear_model import LogisticRegression
    from sklearn.metrics import roc_auc_score

    a, y = activations.detach().cpu().numpy(), labels.detach().cpu().numpy()
    clf = LogisticRegression(**kwargs).fit(a, y)
    return float(roc_auc_score(y, clf.predict_proba(a)[:, 1]))
