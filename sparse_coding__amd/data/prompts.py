"""Indirect-object-identification (IOI) prompt pairs for circuit / ablation studies.

Reference: ``test_datasets/ioi.py`` -- clean/corrupted pairs of the templates
"Then, A and B were working at the L. B decided to give a O to A" (ABB->A) and its
ABA->B swap, with single-token names / places / objects, seeded sampling.

Additions: the answer and distractor token ids are returned with the prompts so
logit-difference metrics need no re-tokenisation (``ioi_logit_diff``), and the
tokenizer is any callable with the HF ``__call__`` -> ``{"input_ids"}`` contract
(``WordTokenizer`` is a dependency-free stand-in for offline tests).
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Dict, List, Sequence, Tuple

import numpy as np
import torch

TEMPLATE_ABB = "Then, {a} and {b} were working at the {place}. {b} decided to give a {obj} to {a}"
TEMPLATE_ABA = "Then, {a} and {b} were working at the {place}. {a} decided to give a {obj} to {b}"

NAMES = ("Alice Amy Andrew Anna Anthony Barbara Ben Betty Brian Carol Charles Chris Daniel David Dennis Donald "
         "Dorothy Edward Emily Emma Eric Frank Gary George Helen Henry Jack Jacob James Jason Jeff Jennifer "
         "Jessica John Joseph Joshua Karen Kate Kevin Larry Laura Linda Lisa Mark Martin Mary Matthew Michael "
         "Nancy Nicole Paul Peter Rachel Richard Robert Ruth Ryan Sam Sarah Scott Sharon Simon Steven Susan "
         "Thomas Tim Tom Victoria Walter William").split()
PLACES = ["cafe", "station", "bridge", "home", "school", "garden", "office"]
OBJECTS = ["ring", "towel", "book", "drink", "key", "bag", "cake"]


class WordTokenizer:
    """Word-level tokenizer: each whitespace-separated word (punctuation split off) is one id."""

    def __init__(self, vocab: Sequence[str] = ()):
        self.vocab: Dict[str, int] = {}
        for w in vocab:
            self._id(w)

    def _id(self, w: str) -> int:
        if w not in self.vocab:
            self.vocab[w] = len(self.vocab)
        return self.vocab[w]

    def _split(self, text: str) -> List[str]:
        out = []
        for w in text.replace(",", " ,").replace(".", " .").split():
            out.append(w)
        return out

    def __call__(self, text):
        if isinstance(text, str):
            return {"input_ids": [self._id(w) for w in self._split(text)]}
        return {"input_ids": [[self._id(w) for w in self._split(t)] for t in text]}


def _single_token(tokenizer, words: Sequence[str]) -> List[str]:
    return [w for w in words if len(tokenizer(" " + w)["input_ids"]) == 1]


@dataclass
class IOIBatch:
    clean: torch.Tensor          # [N, S] token ids
    corrupted: torch.Tensor      # [N, S]
    answer: torch.Tensor         # [N] id of the correct final name (indirect object)
    distractor: torch.Tensor     # [N] id of the subject name
    clean_text: List[str]
    corrupted_text: List[str]


def generate_ioi_dataset(tokenizer: Callable, n_abb_a: int, n_aba_b: int, seed: int = 42) -> IOIBatch:
    """``n_abb_a`` ABB->A clean prompts (corrupted = ABA->B) then ``n_aba_b`` ABA->B prompts
    (corrupted = ABB->A).  Names, places and objects that are not single tokens are dropped
    (places/objects must all be single tokens, as in the reference)."""
    rng = np.random.default_rng(seed)
    names = _single_token(tokenizer, NAMES)
    for group in (PLACES, OBJECTS):
        bad = [w for w in group if len(tokenizer(" " + w)["input_ids"]) != 1]
        if bad:
            raise ValueError(f"not single tokens for this tokenizer: {bad}")
    if len(names) < 2:
        raise ValueError("fewer than two single-token names")
    clean, corrupted, ans, dis = [], [], [], []
    for i in range(n_abb_a + n_aba_b):
        a, b = rng.choice(names, size=2, replace=False)
        place, obj = rng.choice(PLACES), rng.choice(OBJECTS)
        abb = TEMPLATE_ABB.format(a=a, b=b, place=place, obj=obj)
        aba = TEMPLATE_ABA.format(a=a, b=b, place=place, obj=obj)
        if i < n_abb_a:
            clean.append(abb), corrupted.append(aba), ans.append(a), dis.append(b)
        else:
            clean.append(aba), corrupted.append(abb), ans.append(b), dis.append(a)
    # prompts keep the final name; logits at position -2 predict it (ioi_logit_diff)
    ct = torch.tensor(tokenizer(clean)["input_ids"])
    rt = torch.tensor(tokenizer(corrupted)["input_ids"])
    ans_ids = torch.tensor([tokenizer(" " + n)["input_ids"][0] for n in ans])
    dis_ids = torch.tensor([tokenizer(" " + n)["input_ids"][0] for n in dis])
    return IOIBatch(ct, rt, ans_ids, dis_ids, clean, corrupted)


def ioi_logit_diff(logits: torch.Tensor, batch: IOIBatch) -> torch.Tensor:
    """Mean (answer - distractor) logit at the position before the final name."""
    last = logits[:, -2].float()
    idx = torch.arange(last.shape[0], device=last.device)
    return (last[idx, batch.answer.to(last.device)] - last[idx, batch.distractor.to(last.device)]).mean()
