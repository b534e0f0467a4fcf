"""Feature case studies (the reference's notebooks as a library).

Reference: ``minimal_feature_interp.ipynb`` / ``case_studies_loop.ipynb`` /
``interp_notebooks/*.ipynb`` helpers -- ``get_feature_datapoints`` (max / uniform /
random example selection), ``get_neuron_activation``, ``ablate_text`` (per-token
ablation effect), ``ablate_feature_direction`` / ``add_feature_direction``
(steering), ``logit_lens`` / ``visualize_logit_diff`` (direct vocabulary effect),
``prepend_all_tokens_and_get_feature_activation`` (which token before/after a
context maximally activates a feature), ``generate_text`` (greedy generation with an
intervention), ``gini`` / ``select_dict`` (``inter_dict_connections.ipynb``).

Everything runs batched on the device through ``HookedLM`` hooks; rendering is plain
text (``render_activations``), no circuitsvis / IPython dependency.
"""

from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .hooked import HookedLM, lm_loss, tensor_name


# ----------------------------------------------------------------------------- selection
def get_feature_datapoints(feature_acts: torch.Tensor, k: int = 10, setting: str = "max",
                           generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """Indices of ``k`` token positions for one feature's activations [N] (flattened
    (sentence, position)): top-k ("max"), one per activation bin ("uniform", strongest
    first), or random among the positions where it fires ("random")."""
    a = feature_acts.float()
    if setting == "max":
        return torch.argsort(a, descending=True)[:k]
    if setting == "uniform":
        edges = torch.linspace(float(a.min()), float(a.max()), k + 1, device=a.device)
        bins = torch.bucketize(a, edges)
        picks = []
        for b in torch.unique(bins):
            idx = torch.nonzero(bins == b).flatten()
            picks.append(idx[torch.randint(len(idx), (1,), generator=generator, device="cpu").item()])
        return torch.stack(picks).flip(0)
    nz = torch.nonzero(a).flatten()
    return nz[torch.randperm(len(nz), generator=generator)[:k].to(nz.device)]


def unravel(flat_idx: torch.Tensor, seq_len: int) -> List[Tuple[int, int]]:
    return [(int(i) // seq_len, int(i) % seq_len) for i in flat_idx.tolist()]


# ----------------------------------------------------------------------------- activations
@torch.no_grad()
def feature_activations(lm: HookedLM, learned_dict, layer: int, layer_loc: str, tokens: torch.Tensor,
                        feature: Optional[int] = None, basis: str = "dictionary") -> torch.Tensor:
    """Per-token activations [B, S] of one feature (or [B, S, n] for all); ``basis="neuron"``
    returns the raw hook coordinate instead (reference get_neuron_activation)."""
    name = tensor_name(layer, layer_loc)
    _, cache = lm.run_with_cache(tokens, names_filter=[name], return_type=None)
    h = cache[name]
    B, S, D = h.shape
    if basis == "dictionary":
        c = learned_dict.encode(h.reshape(B * S, D).float()).reshape(B, S, -1)
    else:
        c = h.float()
    return c if feature is None else c[..., feature]


@torch.no_grad()
def ablate_tokens(lm: HookedLM, learned_dict, layer: int, layer_loc: str, tokens: torch.Tensor, feature: int,
                  position: int = -1, replacement: int = 0) -> torch.Tensor:
    """Effect of each token up to ``position`` on the feature there (reference ablate_text):
    one batched forward where row i has token i replaced by ``replacement``; returns [pos+1]
    = activation(original) - activation(token i replaced)."""
    toks = tokens.reshape(1, -1).to(lm.device)
    pos = position % toks.shape[1]
    ctx = toks[:, :pos + 1]
    base = feature_activations(lm, learned_dict, layer, layer_loc, ctx, feature)[0, pos]
    batch = ctx.repeat(pos + 1, 1)
    batch[torch.arange(pos + 1), torch.arange(pos + 1)] = replacement
    acts = feature_activations(lm, learned_dict, layer, layer_loc, batch, feature)[:, pos]
    return base - acts


# ----------------------------------------------------------------------------- steering
def _direction(learned_dict, feature: int) -> torch.Tensor:
    return learned_dict.get_learned_dict()[feature]


def add_feature_direction(learned_dict, feature: int, scale: float):
    """Hook: add ``scale`` x the feature's dictionary atom at every position."""
    def hook(t, hook=None):
        return t + scale * _direction(learned_dict, feature).to(t.device, t.dtype)

    return hook


def ablate_feature_direction(learned_dict, feature: int):
    """Hook: remove the feature's contribution (code x atom) at every position."""
    def hook(t, hook=None):
        B, S, D = t.shape
        c = learned_dict.encode(t.reshape(B * S, D).float())[:, feature:feature + 1]
        return t - (c * _direction(learned_dict, feature)[None]).reshape(B, S, D).to(t.dtype)

    return hook


@torch.no_grad()
def logit_diff_under(lm: HookedLM, tokens: torch.Tensor, hook_name: str, hook_fn) -> torch.Tensor:
    """Change of the next-token log-probs [B, S, V] when ``hook_fn`` edits ``hook_name``."""
    base = torch.log_softmax(lm(tokens, return_type="logits").float(), -1)
    edit = torch.log_softmax(lm.run_with_hooks(tokens, [(hook_name, hook_fn)], return_type="logits").float(), -1)
    return edit - base


def top_tokens(scores: torch.Tensor, k: int = 10, detok: Callable[[int], str] = str):
    v_up, i_up = scores.topk(k)
    v_dn, i_dn = scores.topk(k, largest=False)
    return ([(detok(int(i)), float(v)) for i, v in zip(i_up, v_up)],
            [(detok(int(i)), float(v)) for i, v in zip(i_dn, v_dn)])


def logit_lens(lm: HookedLM, learned_dict, feature: int, k: int = 10, detok: Callable[[int], str] = str,
               final_norm: bool = False):
    """Direct effect of the feature's atom on the vocabulary: W_U · atom (optionally through the
    final layer norm's scale) -> top boosted / suppressed tokens."""
    W_U = lm.model.get_output_embeddings().weight.detach().float()  # [V, D]
    atom = _direction(learned_dict, feature).float().to(W_U.device)
    if final_norm:
        ln = getattr(getattr(lm.model, "gpt_neox", None), "final_layer_norm", None) or \
            getattr(getattr(lm.model, "transformer", None), "ln_f", None)
        if ln is not None and getattr(ln, "weight", None) is not None:
            atom = atom * ln.weight.detach().float()
    return top_tokens(W_U @ atom, k, detok)


@torch.no_grad()
def generate_text(lm: HookedLM, tokens: torch.Tensor, n_new: int = 20, fwd_hooks=()) -> torch.Tensor:
    """Greedy continuation [B, S + n_new] with optional interventions in place."""
    toks = tokens.clone()
    for _ in range(n_new):
        logits = lm.run_with_hooks(toks, list(fwd_hooks), return_type="logits")
        toks = torch.cat([toks, logits[:, -1].argmax(-1, keepdim=True).to(toks.device)], dim=1)
    return toks


@torch.no_grad()
def best_context_token(lm: HookedLM, learned_dict, layer: int, layer_loc: str, context: torch.Tensor,
                       feature: int, setting: str = "append", vocab_size: Optional[int] = None,
                       batch_size: int = 512, k: int = 20):
    """Activation of ``feature`` at the last position for every vocabulary token placed
    before ("prepend") or after ("append") ``context`` (reference
    prepend_all_tokens_and_get_feature_activation).  Returns (acts [V], top-k ids up, down)."""
    V = vocab_size or lm.model.get_output_embeddings().weight.shape[0]
    ctx = context.reshape(1, -1).to(lm.device)
    acts = torch.empty(V)
    for s in range(0, V, batch_size):
        ids = torch.arange(s, min(V, s + batch_size), device=lm.device)[:, None]
        rep = ctx.expand(ids.shape[0], -1)
        batch = torch.cat([ids, rep], 1) if setting == "prepend" else torch.cat([rep, ids], 1)
        acts[s:s + ids.shape[0]] = feature_activations(lm, learned_dict, layer, layer_loc, batch, feature)[:, -1].cpu()
    return acts, acts.topk(k).indices, acts.topk(k, largest=False).indices


# ----------------------------------------------------------------------------- rendering / stats
def render_activations(tokens: Sequence[str], acts: Sequence[float], width: int = 8) -> str:
    """One line per token: ``token  ####  0.53`` (bar scaled to the max activation)."""
    m = max([float(a) for a in acts] + [1e-8])
    lines = []
    for t, a in zip(tokens, acts):
        lines.append(f"{t!r:>16} {'#' * int(round(width * max(float(a), 0.0) / m)):<{width}} {float(a):.3f}")
    return "\n".join(lines)


def gini(x: torch.Tensor) -> float:
    """Gini coefficient of a non-negative vector (inter_dict_connections.ipynb)."""
    v = torch.sort(x.flatten().abs().float()).values
    n = v.numel()
    if n == 0 or float(v.sum()) == 0:
        return 0.0
    idx = torch.arange(1, n + 1, dtype=torch.float32, device=v.device)
    return float((2 * (idx * v).sum() / (n * v.sum())) - (n + 1) / n)


def select_dict(learned_dicts, **hparams):
    """First (dict, hparams) whose hyper-parameters match ``hparams`` (float tolerance 1e-6)."""
    for ld, hp in learned_dicts:
        if all(abs(float(hp.get(k, np.nan)) - float(v)) <= 1e-6 * max(1.0, abs(float(v))) if isinstance(v, float)
               else hp.get(k) == v for k, v in hparams.items()):
            return ld, hp
    raise KeyError(f"no dictionary with {hparams}")
