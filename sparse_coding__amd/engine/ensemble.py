"""``FunctionalEnsemble``: many dictionaries trained in one batched pass (eager / oracle path).

Behaviour of reference ``autoencoders/ensemble.py:68-193``: per-model
``(params, buffers)`` dicts are stacked along a leading model axis, gradients
come from ``torch.vmap(torch.func.grad(sig.loss, has_aux=True))`` and the
optimizer update is vmapped too.  ``no_stacking=True`` loops over models for
signatures whose shapes differ per model (top-k with per-model k).

This class is the portable path (CPU, or any signature the fused HIP engine
does not cover).  On MI355X the trainer factory in
``sparse_coding__amd.engine.trainer`` swaps in ``FusedSAEEnsemble`` for the SAE
signatures; both expose ``step_batch``/``unstack``/``state_dict``.
"""

from __future__ import annotations

from typing import List, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor
from torch.utils import _pytree as pytree

from .optim import apply_updates, optim_str_to_func


def construct_stacked_leaf(tensors: Sequence[Tensor], device=None) -> Tensor:
    req = [t.requires_grad for t in tensors]
    if any(req) and not all(req):
        raise RuntimeError("Expected tensors from each model to have the same .requires_grad")
    out = torch.stack(list(tensors)).to(device=device)
    if all(req):
        out = out.detach().requires_grad_()
    return out


def stack_dict(models: list, device=None):
    """Stack a list of identically-structured pytrees along a new leading axis."""
    flat = [pytree.tree_flatten(m) for m in models]
    spec = flat[0][1]
    leaves = [construct_stacked_leaf(ts, device=device) for ts in zip(*[f[0] for f in flat])]
    return pytree.tree_unflatten(leaves, spec)


def unstack_dict(params, n_models: int, device=None) -> list:
    leaves, spec = pytree.tree_flatten(params)
    return [pytree.tree_unflatten([t[i].to(device=device) for t in leaves], spec) for i in range(n_models)]


class FunctionalEnsemble:
    def __init__(self, models, sig, optimizer_func, optimizer_kwargs, device=None, no_stacking=False):
        if isinstance(optimizer_func, str):
            optimizer_func = optim_str_to_func(optimizer_func)
        if device is None:  # fix B#7: infer from the first params dict, not the tuple
            device = next(iter(models[0][0].values())).device
        self.device = device
        self.n_models = len(models)
        params, buffers = zip(*models)
        self.params = stack_dict(list(params), device=device)
        self.buffers = stack_dict(list(buffers), device=device)
        self.sig = sig
        self.no_stacking = no_stacking
        self.optimizer_func = optimizer_func
        self.optimizer_kwargs = dict(optimizer_kwargs)
        self.optimizer = optimizer_func(**self.optimizer_kwargs)
        # vmap may return expanded (stride-0) leaves; materialise so in-place updates work
        self.optim_states = pytree.tree_map(lambda t: t.contiguous().clone(),
                                            torch.vmap(self.optimizer.init)(self.params))
        self.init_functions()

    # ----------------------------------------------------------------- functions
    def init_functions(self):
        grad_fn = torch.func.grad(self.sig.loss, has_aux=True)
        if self.no_stacking:
            def calc_grads(params, buffers, batch):
                grads, auxs = [], []
                for i in range(self.n_models):
                    p = pytree.tree_map(lambda t: t[i], params)
                    b = pytree.tree_map(lambda t: t[i], buffers)
                    g, a = grad_fn(p, b, batch[i])
                    grads.append(g)
                    auxs.append(a)
                return stack_dict(grads), stack_dict(auxs)

            self.calc_grads = calc_grads
        else:
            self.calc_grads = torch.vmap(grad_fn)
        self.update = torch.vmap(self.optimizer.update)

    # ----------------------------------------------------------------- state
    @staticmethod
    def from_state(state_dict):
        self = FunctionalEnsemble.__new__(FunctionalEnsemble)
        for k in ("device", "n_models", "params", "buffers", "sig", "no_stacking", "optimizer_func",
                  "optimizer_kwargs", "optim_states"):
            setattr(self, k, state_dict[k])
        if isinstance(self.optimizer_func, str):
            self.optimizer_func = optim_str_to_func(self.optimizer_func)
        self.optimizer = self.optimizer_func(**self.optimizer_kwargs)
        self.init_functions()
        return self

    def state_dict(self):
        return {
            "device": self.device, "n_models": self.n_models, "params": self.params,
            "buffers": self.buffers, "sig": self.sig, "no_stacking": self.no_stacking,
            "optimizer_func": self.optimizer_func, "optimizer_kwargs": self.optimizer_kwargs,
            "optim_states": self.optim_states,
        }

    def unstack(self, device=None):
        return list(zip(unstack_dict(self.params, self.n_models, device),
                        unstack_dict(self.buffers, self.n_models, device)))

    def to_device(self, device):
        self.device = device
        mv = lambda t: t.to(device)
        self.params = pytree.tree_map(mv, self.params)
        self.buffers = pytree.tree_map(mv, self.buffers)
        self.optim_states = pytree.tree_map(mv, self.optim_states)

    def to_shared_memory(self):
        for tree in (self.params, self.buffers, self.optim_states):
            for t in pytree.tree_leaves(tree):
                t.share_memory_()

    # ----------------------------------------------------------------- training
    def compute_grads(self, minibatches, expand_dims=True):
        """Gradients of every model's loss (no update); returns (grads, (loss_dict, aux))."""
        with torch.no_grad():
            if expand_dims:
                minibatches = minibatches.expand(self.n_models, *minibatches.shape)
            return self.calc_grads(self.params, self.buffers, minibatches)

    def apply_grads(self, grads):
        with torch.no_grad():
            updates, new_states = self.update(grads, self.optim_states)
            # fix B#6: actually write the new optimizer state back
            for old, new in zip(pytree.tree_leaves(self.optim_states), pytree.tree_leaves(new_states)):
                old.copy_(new)
            apply_updates(self.params, updates)

    def step_batch(self, minibatches, expand_dims=True):
        grads, (loss, aux) = self.compute_grads(minibatches, expand_dims)
        self.apply_grads(grads)
        return loss, aux

    def to_learned_dicts(self, device="cpu"):
        return [self.sig.to_learned_dict(p, b) for p, b in self.unstack(device)]
