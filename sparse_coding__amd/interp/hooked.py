"""``HookedLM``: named hook points over a HuggingFace GPT-NeoX / GPT-2 model.

The reference drives TransformerLens (``HookedTransformer.run_with_hooks`` /
``run_with_cache``, ``standard_metrics.py:36-112, 222-250``); TransformerLens is
not available here, so this wrapper exposes the same surface -- TL hook names,
``fwd_hooks=[(name, fn)]`` with ``fn(tensor, hook=None) -> tensor | None``,
``return_type="loss" | "logits" | None`` and ``run_with_cache(names_filter=...)`` --
on top of ``torch.nn.Module`` forward hooks of the HF model built by
``data.harvest.build_model``.

Hook names (``L`` = layer index):

* ``blocks.L.hook_resid_post``  -- block output (residual stream), ``[B, S, d_model]``
* ``blocks.L.mlp.hook_post``    -- post-activation MLP hidden, ``[B, S, d_mlp]``
* ``blocks.L.hook_mlp_out``     -- MLP output, ``[B, S, d_model]``
* ``blocks.L.attn.hook_z``      -- concatenated head outputs, ``[B, S, n_heads * d_head]``
"""

from __future__ import annotations

import re
from contextlib import contextmanager
from typing import Callable, Dict, Iterable, List, Optional, Sequence, Tuple, Union

import torch
import torch.nn.functional as F

from ..data.harvest import _blocks, _hook_module

HookFn = Callable[..., Optional[torch.Tensor]]
_NAME = re.compile(r"^blocks\.(\d+)\.(hook_resid_post|mlp\.hook_post|hook_mlp_out|attn\.hook_z)$")
_LOC = {"hook_resid_post": "residual", "mlp.hook_post": "mlp", "hook_mlp_out": "mlpout", "attn.hook_z": "attn"}


def tensor_name(layer: int, layer_loc: str) -> str:
    """(layer, residual|mlp|mlpout|attn) -> hook name (reference get_model_tensor_name)."""
    return {"residual": f"blocks.{layer}.hook_resid_post", "mlp": f"blocks.{layer}.mlp.hook_post",
            "mlpout": f"blocks.{layer}.hook_mlp_out", "attn": f"blocks.{layer}.attn.hook_z"}[layer_loc]


def parse_name(name: str) -> Tuple[int, str]:
    m = _NAME.match(name)
    if not m:
        raise ValueError(f"unknown hook point {name!r}")
    return int(m.group(1)), _LOC[m.group(2)]


class HookedLM:
    def __init__(self, model, tokenizer=None):
        self.model = model
        self.tokenizer = tokenizer
        blocks, self.arch = _blocks(model)
        self.n_layers = len(blocks)

    @classmethod
    def from_config(cls, model_name: str, device="cuda", dtype=torch.float32, seed: int = 0, pretrained_dir: str = ""):
        from ..data.harvest import build_model

        return cls(build_model(model_name, device=device, dtype=dtype, seed=seed, pretrained_dir=pretrained_dir))

    @property
    def device(self):
        return next(self.model.parameters()).device

    # ------------------------------------------------------------------ hook plumbing
    def _register(self, name: str, fn: HookFn):
        layer, loc = parse_name(name)
        mod, use_input = _hook_module(self.model, layer, loc)

        class _Hook:  # TL passes a HookPoint; functions here only ever read .name
            pass

        hp = _Hook()
        hp.name = name
        if use_input:
            def pre(module, args):
                out = fn(args[0], hook=hp)
                if out is not None:
                    return (out,) + tuple(args[1:])
                return None

            return mod.register_forward_pre_hook(pre)

        def post(module, args, output):
            t = output[0] if isinstance(output, tuple) else output
            out = fn(t, hook=hp)
            if out is None:
                return None
            return (out,) + tuple(output[1:]) if isinstance(output, tuple) else out

        return mod.register_forward_hook(post)

    @contextmanager
    def hooks(self, fwd_hooks: Sequence[Tuple[str, HookFn]] = ()):
        handles = [self._register(n, f) for n, f in fwd_hooks]
        try:
            yield self
        finally:
            for h in handles:
                h.remove()

    # ------------------------------------------------------------------ forward API
    def _forward(self, tokens: torch.Tensor, return_type: Optional[str]):
        tokens = tokens.to(self.device)
        logits = self.model(input_ids=tokens).logits
        if return_type == "logits":
            return logits
        if return_type == "loss":
            return lm_loss(logits, tokens)
        if return_type == "both":
            return logits, lm_loss(logits, tokens)
        return None

    @torch.no_grad()
    def __call__(self, tokens, return_type: Optional[str] = "logits"):
        return self._forward(tokens, return_type)

    @torch.no_grad()
    def run_with_hooks(self, tokens, fwd_hooks: Sequence[Tuple[str, HookFn]] = (), return_type: Optional[str] = "logits"):
        with self.hooks(fwd_hooks):
            return self._forward(tokens, return_type)

    @torch.no_grad()
    def run_with_cache(self, tokens, names_filter: Union[None, str, Sequence[str], Callable[[str], bool]] = None,
                       fwd_hooks: Sequence[Tuple[str, HookFn]] = (), return_type: Optional[str] = "logits"):
        names = self._names(names_filter)
        cache: Dict[str, torch.Tensor] = {}

        def saver(t, hook=None):
            cache[hook.name] = t.detach().clone()

        with self.hooks(list(fwd_hooks) + [(n, saver) for n in names]):
            out = self._forward(tokens, return_type)
        return out, cache

    def _names(self, names_filter) -> List[str]:
        all_names = [tensor_name(L, loc) for L in range(self.n_layers) for loc in ("residual", "mlp", "mlpout", "attn")]
        if names_filter is None:
            return all_names
        if isinstance(names_filter, str):
            return [names_filter]
        if callable(names_filter):
            return [n for n in all_names if names_filter(n)]
        return list(names_filter)


def lm_loss(logits: torch.Tensor, tokens: torch.Tensor, per_token: bool = False) -> torch.Tensor:
    """Mean next-token cross-entropy (TransformerLens ``return_type="loss"``)."""
    lp = F.log_softmax(logits[:, :-1].float(), dim=-1)
    nll = -lp.gather(-1, tokens[:, 1:, None].to(lp.device)).squeeze(-1)
    return nll if per_token else nll.mean()
