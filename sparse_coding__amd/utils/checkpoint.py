"""Checkpoint formats.

1. **Reference-compatible** ``learned_dicts.pt``:
   ``torch.save(list[tuple[LearnedDict, dict]])`` with classes addressed as
   ``autoencoders.learned_dict.TiedSAE`` etc. (reference ``big_sweep.py:424``,
   ``basic_l1_sweep.py:113``).  ``load_learned_dicts`` reads the reference's own
   files with ``torch.load(weights_only=True)`` plus an allow-list of exactly the
   dictionary classes (nothing else in the file can execute); ``save_learned_dicts``
   writes the same layout by re-classing native objects to the ``autoencoders.*``
   aliases.
2. **Native training checkpoint** (the reference never saves optimizer state, so it
   cannot resume): parameters, Adam moments, step counter, RNG states,
   data cursor and the config, as a dict of tensors and plain values -- also
   loadable with ``weights_only=True``.
"""

from __future__ import annotations

import copy
import importlib
import os
from typing import Any, Dict, Iterable, List, Tuple

import torch

_ALIAS_MODULES = [
    "autoencoders.learned_dict", "autoencoders.fista", "autoencoders.topk_encoder", "autoencoders.pca",
    "autoencoders.sae_ensemble", "autoencoders.ica", "autoencoders.nmf", "autoencoders.direct_coef_search",
    "autoencoders.residual_denoising_autoencoder", "autoencoders.mlp_tests",
]


def _alias_classes() -> Dict[type, type]:
    """native class -> alias class (the alias is a subclass living under ``autoencoders.*``)."""
    from ..models.learned_dict import LearnedDict

    out = {}
    for mod_name in _ALIAS_MODULES:
        mod = importlib.import_module(mod_name)
        for name in dir(mod):
            obj = getattr(mod, name)
            if isinstance(obj, type) and issubclass(obj, LearnedDict) and obj.__module__ == mod_name:
                out[obj.__mro__[1]] = obj
    return out


def _safe_globals() -> List[type]:
    classes = list(_alias_classes().values())
    from ..models import learned_dict as ld

    natives = [getattr(ld, n) for n in ("Identity", "IdentityReLU", "RandomDict", "UntiedSAE", "TiedSAE",
                                        "ReverseSAE", "AddedNoise", "Rotation")]
    return classes + natives


def load_learned_dicts(path: str, map_location="cpu") -> List[Tuple[Any, dict]]:
    """Load a ``learned_dicts.pt`` (reference or ours) without executing pickled code."""
    with torch.serialization.safe_globals(_safe_globals()):
        obj = torch.load(path, map_location=map_location, weights_only=True)
    if isinstance(obj, tuple):
        obj = [obj]
    for ld, _ in obj:
        if hasattr(ld, "initialize_missing"):
            ld.initialize_missing()  # old pickles may lack centering (reference learned_dict.py:156-164)
    return obj


def to_compat(ld):
    """Shallow copy of ``ld`` whose class is the ``autoencoders.*`` alias (reference pickle path)."""
    alias = _alias_classes().get(type(ld))
    if alias is None:
        return ld
    out = copy.copy(ld)
    out.__class__ = alias
    return out


def save_learned_dicts(learned_dicts: Iterable[Tuple[Any, dict]], path: str, compat: bool = True):
    """Write ``list[(LearnedDict, hparams)]``; with ``compat`` the file matches the reference layout."""
    items = []
    for ld, hp in learned_dicts:
        if hasattr(ld, "to_device"):
            ld = copy.copy(ld)
            ld.to_device("cpu")
        items.append((to_compat(ld) if compat else ld, dict(hp)))
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = path + ".tmp"
    torch.save(items, tmp)
    os.replace(tmp, path)


# ----------------------------------------------------------------------------- native training state
def rng_state() -> Dict[str, Any]:
    st = {"torch_cpu": torch.get_rng_state()}
    if torch.cuda.is_available():
        st["torch_cuda"] = torch.cuda.get_rng_state_all()
    return st


def set_rng_state(st: Dict[str, Any]):
    torch.set_rng_state(st["torch_cpu"])
    if "torch_cuda" in st and torch.cuda.is_available():
        torch.cuda.set_rng_state_all(st["torch_cuda"])


def save_training_state(path: str, trainer_state: Dict[str, Any], extra: Dict[str, Any] | None = None):
    """Atomic write of a resumable checkpoint: tensors + plain python values only."""
    payload = {"format": "sparse_coding__amd/train-v1", "trainer": _to_cpu(trainer_state), "rng": rng_state(),
               "extra": extra or {}}
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = path + ".tmp"
    torch.save(payload, tmp)
    os.replace(tmp, path)


def load_training_state(path: str, map_location="cpu") -> Dict[str, Any]:
    payload = torch.load(path, map_location=map_location, weights_only=True)
    if payload.get("format") != "sparse_coding__amd/train-v1":
        raise ValueError(f"{path} is not a sparse_coding__amd training checkpoint")
    return payload


def _to_cpu(obj):
    if torch.is_tensor(obj):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, tuple) and hasattr(obj, "_fields"):
        # optimizer NamedTuples -> plain lists: weights_only loading admits no custom classes,
        # and restoring walks pytree leaves, whose order is the field order either way
        return [_to_cpu(v) for v in obj]
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    return obj
