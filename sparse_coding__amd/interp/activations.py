"""Feature-activation datasets: per-fragment, per-token dictionary activations.

Reference: ``interpret.py:82-212`` (``make_feature_activation_dataset``) and
``:215-253`` (``get_df``): 50k random 64-token fragments (one per document), the
LM activation at (layer, loc) encoded by the dictionary, stored as a pandas table
with a ``feature_i_max`` column and 64 ``feature_i_activation_j`` columns per feature.

MI355X design: fragments run through the LM in large batches; the activations are
encoded on the device and written straight into preallocated fp16 tensors
``acts [F, L, n_feats]`` / ``maxes [F, n_feats]`` (no per-fragment Python loop, no
wide DataFrame).  The dataset saves as a dict of tensors (loads with
``weights_only=True``); ``to_dataframe`` produces the reference's column layout
when a pandas table is wanted.
"""

from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Callable, Iterator, List, Optional, Sequence

import numpy as np
import torch

from .hooked import HookedLM, tensor_name

FRAGMENT_LEN = 64
MAX_FRAGMENTS = 50000


@dataclass
class FeatureActivationDataset:
    token_ids: torch.Tensor     # [F, L] int32
    acts: torch.Tensor          # [F, L, n] fp16
    maxes: torch.Tensor         # [F, n] fp16
    token_strs: Optional[List[List[str]]] = None

    @property
    def n_feats(self) -> int:
        return self.acts.shape[-1]

    def __len__(self):
        return self.acts.shape[0]

    def save(self, path: str):
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        torch.save({"token_ids": self.token_ids, "acts": self.acts, "maxes": self.maxes,
                    "token_strs": self.token_strs}, path)

    @classmethod
    def load(cls, path: str) -> "FeatureActivationDataset":
        d = torch.load(path, weights_only=True)
        return cls(d["token_ids"], d["acts"], d["maxes"], d.get("token_strs"))

    def top_fragments(self, feat: int, k: int) -> torch.Tensor:
        """Indices of the ``k`` fragments with the largest max activation of ``feat``."""
        return torch.topk(self.maxes[:, feat].float(), min(k, len(self))).indices

    def random_active_fragments(self, feat: int, k: int, generator: Optional[torch.Generator] = None
                                ) -> Optional[torch.Tensor]:
        """``k`` random fragments on which ``feat`` fires at all; None if fewer exist."""
        active = torch.nonzero(self.maxes[:, feat] > 0).flatten()
        if active.numel() < k:
            return None
        return active[torch.randperm(active.numel(), generator=generator)[:k]]

    def to_dataframe(self):
        """Reference column layout (``fragment_token_ids``, ``feature_i_max``,
        ``feature_i_activation_j``)."""
        import pandas as pd

        F, L, n = self.acts.shape
        cols = {"fragment_token_ids": [r.tolist() for r in self.token_ids]}
        if self.token_strs is not None:
            cols["fragment_token_strs"] = self.token_strs
        df = pd.DataFrame(cols)
        maxes = pd.DataFrame(self.maxes.float().numpy(), columns=[f"feature_{i}_max" for i in range(n)])
        acts = pd.DataFrame(self.acts.reshape(F, L * n).float().numpy(),  # column j*n + i
                            columns=[f"feature_{i}_activation_{j}" for j in range(L) for i in range(n)])
        return pd.concat([df, maxes, acts], axis=1)


def random_fragments(token_docs: Iterator[torch.Tensor], n: int, fragment_len: int = FRAGMENT_LEN,
                     rng: Optional[np.random.Generator] = None, random_start: bool = True) -> torch.Tensor:
    """One random ``fragment_len`` window per document (reference :136-157); documents shorter
    than a fragment are skipped."""
    rng = rng or np.random.default_rng(0)
    out = []
    for doc in token_docs:
        doc = doc.flatten()
        if doc.numel() < fragment_len:
            continue
        s = int(rng.integers(0, doc.numel() - fragment_len + 1)) if random_start else 0
        out.append(doc[s:s + fragment_len])
        if len(out) >= n:
            break
    return torch.stack(out)


@torch.no_grad()
def make_feature_activation_dataset(lm: HookedLM, learned_dict, layer: int, layer_loc: str,
                                    fragments: torch.Tensor, max_features: int = 0, batch_size: int = 256,
                                    tokenizer=None, store_device="cpu") -> FeatureActivationDataset:
    """Encode every fragment's activations at (layer, layer_loc) with ``learned_dict``."""
    dev = lm.device
    learned_dict.to_device(dev)
    name = tensor_name(layer, layer_loc)
    n_all = learned_dict.get_learned_dict().shape[0]
    n = min(max_features, n_all) if max_features else n_all
    F, L = fragments.shape
    acts = torch.empty(F, L, n, dtype=torch.float16, device=store_device)
    maxes = torch.empty(F, n, dtype=torch.float16, device=store_device)
    for i in range(0, F, batch_size):
        toks = fragments[i:i + batch_size].to(dev)
        _, cache = lm.run_with_cache(toks, names_filter=[name], return_type=None)
        h = cache[name]
        b = h.shape[0]
        c = learned_dict.encode(h.reshape(b * L, -1).float())[:, :n].reshape(b, L, n)
        acts[i:i + b] = c.to(store_device, torch.float16)
        maxes[i:i + b] = c.max(dim=1).values.to(store_device, torch.float16)
    strs = None
    if tokenizer is not None and hasattr(tokenizer, "convert_ids_to_tokens"):
        strs = [tokenizer.convert_ids_to_tokens(r.tolist()) for r in fragments]
    return FeatureActivationDataset(fragments.to(torch.int32).cpu(), acts, maxes, strs)


def get_dataset(learned_dict, lm: HookedLM, layer: int, layer_loc: str, n_feats: int, save_loc: str,
                fragments: Callable[[], torch.Tensor], force_refresh: bool = False, **kw) -> FeatureActivationDataset:
    """Cached ``make_feature_activation_dataset`` (reference get_df)."""
    path = os.path.join(save_loc, "activation_dataset.pt")
    if os.path.exists(path) and not force_refresh:
        ds = FeatureActivationDataset.load(path)
        if ds.n_feats >= n_feats:
            return ds
    ds = make_feature_activation_dataset(lm, learned_dict, layer, layer_loc, fragments(), max_features=n_feats, **kw)
    ds.save(path)
    return ds
