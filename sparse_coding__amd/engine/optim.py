"""Functional optimizers for stacked ensembles (replaces the reference's torchopt dependency).

Semantics follow torchopt 0.7.1 (reference ``requirements.txt:132``) as used by
``autoencoders/ensemble.py:25-31, 94-95, 123``: an optimizer is a pair of pure
functions ``init(params) -> state`` and ``update(grads, state) -> (updates, state)``
so that both can be ``torch.vmap``-ed over the model axis, plus
``apply_updates(params, updates)`` which adds the updates in place.

Adam: ``m <- b1 m + (1-b1) g``; ``v <- b2 v + (1-b2) g^2``;
``u = -lr * (m / (1 - b1^t)) / (sqrt(v / (1 - b2^t) + eps_root) + eps)``.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Callable, NamedTuple

import torch
from torch.utils import _pytree as pytree


class AdamState(NamedTuple):
    mu: Any
    nu: Any
    count: torch.Tensor


class SGDState(NamedTuple):
    momentum: Any


@dataclass(frozen=True)
class FunctionalOptimizer:
    name: str
    init: Callable
    update: Callable
    hparams: dict


def adam(lr=1e-3, betas=(0.9, 0.999), eps=1e-8, eps_root=0.0, weight_decay=0.0):
    b1, b2 = betas

    def init(params):
        zeros = pytree.tree_map(torch.zeros_like, params)
        return AdamState(zeros, pytree.tree_map(torch.zeros_like, params),
                         torch.zeros((), dtype=torch.float32, device=_first(params).device))

    def update(grads, state):
        count = state.count + 1
        if weight_decay:
            raise NotImplementedError("weight decay needs params; use AdamW via trainer")
        mu = pytree.tree_map(lambda m, g: b1 * m + (1 - b1) * g, state.mu, grads)
        nu = pytree.tree_map(lambda v, g: b2 * v + (1 - b2) * g * g, state.nu, grads)
        bc1 = 1 - b1 ** count
        bc2 = 1 - b2 ** count
        updates = pytree.tree_map(
            lambda m, v: -lr * (m / bc1) / (torch.sqrt(v / bc2 + eps_root) + eps), mu, nu)
        return updates, AdamState(mu, nu, count)

    return FunctionalOptimizer("adam", init, update, dict(lr=lr, betas=betas, eps=eps, eps_root=eps_root))


def sgd(lr=1e-3, momentum=0.0, nesterov=False):
    def init(params):
        return SGDState(pytree.tree_map(torch.zeros_like, params))

    def update(grads, state):
        if momentum == 0.0:
            return pytree.tree_map(lambda g: -lr * g, grads), state
        buf = pytree.tree_map(lambda b, g: momentum * b + g, state.momentum, grads)
        if nesterov:
            upd = pytree.tree_map(lambda b, g: -lr * (g + momentum * b), buf, grads)
        else:
            upd = pytree.tree_map(lambda b: -lr * b, buf)
        return upd, SGDState(buf)

    return FunctionalOptimizer("sgd", init, update, dict(lr=lr, momentum=momentum, nesterov=nesterov))


def apply_updates(params, updates):
    """In-place ``p += u`` over matching pytrees (torchopt.apply_updates, inplace=True)."""
    for p, u in zip(pytree.tree_leaves(params), pytree.tree_leaves(updates)):
        p.add_(u)
    return params


def optim_str_to_func(name: str):
    """Reference ``autoencoders/ensemble.py:25-31``."""
    if name == "adam":
        return adam
    if name == "sgd":
        return sgd
    raise ValueError(f"Unknown optimizer string: {name}")


def _first(tree):
    leaves = pytree.tree_leaves(tree)
    return leaves[0]
