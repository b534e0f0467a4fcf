"""Automatic feature interpretation: explain a feature from its top-activating
fragments, simulate activations from the explanation, score by correlation.

Reference: ``interpret.py:256-700`` -- OpenAI ``neuron_explainer``
(``TokenActivationPairExplainer`` + ``ExplanationNeuronSimulator``, gpt-4 /
text-davinci), top-10 + random-10 fragments per feature, interleaved train/valid
splits, correlation scores (all / top-only / random-only) written to
``feature_{n}/explanation.txt``, then ``read_scores`` for plots, and job fan-out
over GPUs.

Neither ``neuron_explainer`` nor network access exists here, so the LLM calls sit
behind two small protocols:

* ``Explainer.explain(records, max_activation) -> str``
* ``Simulator.simulate(explanation, tokens) -> list[float]`` (one value per token)

``OpenAICompatibleExplainer/Simulator`` talk to any chat-completions endpoint
(``SC_INTERP_ENDPOINT`` / ``SC_INTERP_API_KEY``; they refuse to run without one) and
``TokenStatsExplainer`` / ``TokenListSimulator`` are deterministic offline
stand-ins (explanation = the feature's top tokens; simulation = 1 on those tokens)
that exercise the whole pipeline.  Records/scores are stored as JSON, never pickle.
"""

from __future__ import annotations

import json
import os
from dataclasses import asdict, dataclass, field
from typing import Dict, List, Optional, Protocol, Sequence, Tuple

import numpy as np
import torch

from .activations import FeatureActivationDataset

EXAMPLES_PER_SPLIT = 5
N_SPLITS = 2
TOTAL_EXAMPLES = EXAMPLES_PER_SPLIT * N_SPLITS


@dataclass
class ActivationRecord:
    tokens: List[str]
    activations: List[float]


@dataclass
class FeatureRecord:
    feature: int
    top: List[ActivationRecord]
    random: List[ActivationRecord]

    def _split(self, recs, i):
        return recs[i::N_SPLITS]  # interleaved splits: every split sees strong and weak top examples

    def train_records(self) -> List[ActivationRecord]:
        return self._split(self.top, 0) + self._split(self.random, 0)

    def valid_records(self) -> Tuple[List[ActivationRecord], List[ActivationRecord]]:
        return self._split(self.top, 1), self._split(self.random, 1)


class Explainer(Protocol):
    def explain(self, records: Sequence[ActivationRecord], max_activation: float) -> str: ...


class Simulator(Protocol):
    def simulate(self, explanation: str, tokens: Sequence[str]) -> List[float]: ...


# ----------------------------------------------------------------------------- offline stand-ins
class TokenStatsExplainer:
    """Explanation = the ``k`` tokens with the largest mean activation in the records."""

    def __init__(self, k: int = 5):
        self.k = k

    def explain(self, records, max_activation):
        tot: Dict[str, float] = {}
        cnt: Dict[str, int] = {}
        for r in records:
            for t, a in zip(r.tokens, r.activations):
                tot[t] = tot.get(t, 0.0) + float(a)
                cnt[t] = cnt.get(t, 0) + 1
        best = sorted(tot, key=lambda t: -tot[t] / cnt[t])[: self.k]
        return "tokens: " + " | ".join(best)


class TokenListSimulator:
    """Predicts 1 on tokens listed in a ``TokenStatsExplainer`` explanation, else 0."""

    def simulate(self, explanation, tokens):
        listed = set(explanation.split("tokens: ", 1)[-1].split(" | "))
        return [1.0 if t in listed else 0.0 for t in tokens]


# ----------------------------------------------------------------------------- LLM endpoint
class _Endpoint:
    def __init__(self, model: str, endpoint: Optional[str] = None, api_key: Optional[str] = None, timeout: float = 60):
        self.model = model
        self.endpoint = endpoint or os.environ.get("SC_INTERP_ENDPOINT", "")
        self.api_key = api_key or os.environ.get("SC_INTERP_API_KEY", "")
        self.timeout = timeout
        if not self.endpoint:
            raise RuntimeError("no explainer endpoint configured (set SC_INTERP_ENDPOINT); "
                               "use TokenStatsExplainer/TokenListSimulator offline")

    def chat(self, prompt: str) -> str:
        import requests

        r = requests.post(self.endpoint, timeout=self.timeout,
                          headers={"Authorization": f"Bearer {self.api_key}"} if self.api_key else {},
                          json={"model": self.model, "messages": [{"role": "user", "content": prompt}],
                                "temperature": 0})
        r.raise_for_status()
        return r.json()["choices"][0]["message"]["content"]


def _fmt_records(records, max_activation):
    lines = []
    for r in records:
        scaled = [int(round(10 * a / max_activation)) if max_activation > 0 else 0 for a in r.activations]
        lines.append("\n".join(f"{t}\t{s}" for t, s in zip(r.tokens, scaled)))
    return "\n<end>\n".join(lines)


class OpenAICompatibleExplainer(_Endpoint):
    def explain(self, records, max_activation):
        prompt = ("Each block lists tokens with a feature's activation (0-10). In one short phrase, "
                  "what does the feature respond to?\n\n" + _fmt_records(records, max_activation))
        return self.chat(prompt).strip()


class OpenAICompatibleSimulator(_Endpoint):
    def simulate(self, explanation, tokens):
        prompt = (f"A feature responds to: {explanation}\nFor each token below output an integer 0-10, one per "
                  "line, nothing else.\n" + "\n".join(tokens))
        vals = []
        for line in self.chat(prompt).splitlines():
            try:
                vals.append(float(line.strip().split()[-1]))
            except (ValueError, IndexError):
                continue
        return (vals + [0.0] * len(tokens))[: len(tokens)]


# ----------------------------------------------------------------------------- scoring
def correlation_score(true: Sequence[Sequence[float]], pred: Sequence[Sequence[float]]) -> float:
    """Pearson correlation over all tokens of all records (neuron_explainer's ev-correlation)."""
    t = np.concatenate([np.asarray(x, dtype=np.float64) for x in true]) if true else np.zeros(0)
    p = np.concatenate([np.asarray(x, dtype=np.float64) for x in pred]) if pred else np.zeros(0)
    if t.size < 2 or t.std() == 0 or p.std() == 0:
        return 0.0
    return float(np.corrcoef(t, p)[0, 1])


def _records(ds: FeatureActivationDataset, feat: int, idx: torch.Tensor, detok) -> List[ActivationRecord]:
    out = []
    for i in idx.tolist():
        toks = ds.token_strs[i] if ds.token_strs is not None else [detok(t) for t in ds.token_ids[i].tolist()]
        out.append(ActivationRecord(list(toks), ds.acts[i, :, feat].float().tolist()))
    return out


def feature_record(ds: FeatureActivationDataset, feat: int, generator: Optional[torch.Generator] = None,
                   detok=str) -> Optional[FeatureRecord]:
    """Top-``TOTAL_EXAMPLES`` fragments by max activation plus as many random fragments on which
    the feature fires (reference :263-321); None when too few fragments activate it."""
    rnd = ds.random_active_fragments(feat, TOTAL_EXAMPLES, generator)
    if rnd is None:
        return None
    return FeatureRecord(feat, _records(ds, feat, ds.top_fragments(feat, TOTAL_EXAMPLES), detok),
                         _records(ds, feat, rnd, detok))


def interpret_feature(rec: FeatureRecord, explainer: Explainer, simulator: Simulator) -> Dict[str, float]:
    train = rec.train_records()
    max_act = max((max(r.activations) for r in train), default=0.0)
    explanation = explainer.explain(train, max_act)
    top_v, rnd_v = rec.valid_records()
    sims_top = [simulator.simulate(explanation, r.tokens) for r in top_v]
    sims_rnd = [simulator.simulate(explanation, r.tokens) for r in rnd_v]
    true_top = [r.activations for r in top_v]
    true_rnd = [r.activations for r in rnd_v]
    return {"explanation": explanation,
            "score": correlation_score(true_top + true_rnd, sims_top + sims_rnd),
            "top_only_score": correlation_score(true_top, sims_top),
            "random_only_score": correlation_score(true_rnd, sims_rnd)}


def interpret(ds: FeatureActivationDataset, save_folder: str, n_feats_to_explain: int, explainer: Explainer,
              simulator: Simulator, seed: int = 0, detok=str, explainer_name: str = "", simulator_name: str = ""
              ) -> Dict[int, Dict[str, float]]:
    """Explain + score features ``0..n-1``; one ``feature_{n}/`` folder each (skips existing)."""
    g = torch.Generator().manual_seed(seed)
    results = {}
    for f in range(min(n_feats_to_explain, ds.n_feats)):
        folder = os.path.join(save_folder, f"feature_{f}")
        if os.path.exists(folder):
            continue
        rec = feature_record(ds, f, g, detok)
        os.makedirs(folder, exist_ok=True)  # placeholder for skipped features too (reference :309-312)
        if rec is None:
            continue
        res = interpret_feature(rec, explainer, simulator)
        results[f] = res
        with open(os.path.join(folder, "explanation.txt"), "w") as fh:
            fh.write(f"{res['explanation']}\nScore: {res['score']:.2f}\n"
                     f"Explainer model: {explainer_name or type(explainer).__name__}\n"
                     f"Simulator model: {simulator_name or type(simulator).__name__}\n"
                     f"Top only score: {res['top_only_score']:.2f}\n"
                     f"Random only score: {res['random_only_score']:.2f}\n")
        with open(os.path.join(folder, "record.json"), "w") as fh:
            json.dump({"feature": f, "top": [asdict(r) for r in rec.top], "random": [asdict(r) for r in rec.random],
                       **res}, fh)
    return results


# ----------------------------------------------------------------------------- reading results
def get_score(lines: List[str], mode: str) -> float:
    if mode == "top":
        return float(lines[-3].split(" ")[-1])
    if mode == "random":
        return float(lines[-2].split(" ")[-1])
    if mode == "top_random":
        return float([l for l in lines if l.startswith("Score: ")][0].split(" ")[1])
    raise ValueError(f"Unknown mode: {mode}")


def read_transform_scores(transform_loc: str, score_mode: str) -> Tuple[List[int], List[float]]:
    idx, scores = [], []
    for name in sorted(os.listdir(transform_loc)):
        path = os.path.join(transform_loc, name, "explanation.txt")
        if not name.startswith("feature_") or not os.path.exists(path):
            continue
        with open(path) as fh:
            scores.append(get_score(fh.read().split("\n"), score_mode))
        idx.append(int(name.split("_")[1]))
    return idx, scores


def read_scores(results_folder: str, score_mode: str = "top") -> Dict[str, Tuple[List[int], List[float]]]:
    assert score_mode in ("top", "random", "top_random")
    names = sorted(t for t in os.listdir(results_folder) if os.path.isdir(os.path.join(results_folder, t)))
    if "sparse_coding" in names:
        names.remove("sparse_coding")
        names.insert(0, "sparse_coding")
    out = {}
    for t in names:
        i, s = read_transform_scores(os.path.join(results_folder, t), score_mode)
        if i:
            out[t] = (i, s)
    return out


def make_tag_name(hparams: Dict) -> str:
    tag = ""
    if "tied" in hparams:
        tag += f"tied_{hparams['tied']}"
    if "dict_size" in hparams:
        tag += f"dict_size_{hparams['dict_size']}"
    if "l1_alpha" in hparams:
        tag += f"l1_alpha_{hparams['l1_alpha']:.2}"
    if "bias_decay" in hparams:
        tag += "0.0" if hparams["bias_decay"] == 0 else f"{hparams['bias_decay']:.1}"
    return tag


def parse_folder_name(folder_name: str) -> Tuple[str, str, int, float, str]:
    """``tied_residual_l5_r8[_extra]`` -> (tied, loc, layer, ratio, extra); r0 means 0.5."""
    tied, loc, layer_s, ratio_s, *extra = folder_name.split("_")
    ratio = float(ratio_s[1:])
    return tied, loc, int(layer_s[1:]), ratio if ratio else 0.5, "_".join(extra)
