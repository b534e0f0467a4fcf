"""Activation harvester: transformer forward -> hook tensor -> HBM ring / chunk files.

Reference: ``activation_dataset.py:39-467`` (TransformerLens ``run_with_cache`` on
Pythia / GPT-2, fp16 chunks of 2 GiB, 4 x 256-token batches).  Differences, all
MI355X-driven:

* models are HuggingFace ``transformers`` classes built from the published
  architecture configs (Pythia-70m/410m/1.4b GPT-NeoX, GPT-2-small) with random
  init -- there is no network for checkpoints (``load_pretrained`` loads a local
  directory when one exists);
* the forward runs in bf16 and stops after the deepest hooked layer;
* hook outputs go straight into the device ``DeviceRing`` (no host round trip) and
  optionally to reference-format ``{i}.pt`` fp16 chunks;
* ``attn`` hooks the concatenated head outputs (fix B#13: the reference returned the
  residual stream while sizing the buffer d_head * n_heads);
* every chunk holds exactly ``rows_per_chunk`` rows (fix B#26).

Token sources: a Zipf-distributed synthetic stream (default, offline), token-id
files, or local text with a local tokenizer (``chunk_and_tokenize``).
"""

from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Callable, Dict, Iterable, Iterator, List, Optional, Sequence, Tuple

import torch

MODEL_BATCH_SIZE = 4
CHUNK_SIZE_GB = 2.0
MAX_SENTENCE_LEN = 256

# Published architecture hyper-parameters (HF config.json of the named checkpoints).
MODEL_CONFIGS: Dict[str, Dict] = {
    "pythia-70m": dict(arch="gpt_neox", hidden_size=512, num_hidden_layers=6, num_attention_heads=8,
                       intermediate_size=2048, vocab_size=50304, rotary_pct=0.25, max_position_embeddings=2048),
    "pythia-160m": dict(arch="gpt_neox", hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                        intermediate_size=3072, vocab_size=50304, rotary_pct=0.25, max_position_embeddings=2048),
    "pythia-410m": dict(arch="gpt_neox", hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
                        intermediate_size=4096, vocab_size=50304, rotary_pct=0.25, max_position_embeddings=2048),
    "pythia-1.4b": dict(arch="gpt_neox", hidden_size=2048, num_hidden_layers=24, num_attention_heads=16,
                        intermediate_size=8192, vocab_size=50304, rotary_pct=0.25, max_position_embeddings=2048),
    "gpt2": dict(arch="gpt2", n_embd=768, n_layer=12, n_head=12, vocab_size=50257, n_positions=1024),
    "gpt2-medium": dict(arch="gpt2", n_embd=1024, n_layer=24, n_head=16, vocab_size=50257, n_positions=1024),
}
_ALIASES = {"pythia-70m-deduped": "pythia-70m", "EleutherAI/pythia-70m-deduped": "pythia-70m",
            "EleutherAI/pythia-70m": "pythia-70m", "pythia-410m-deduped": "pythia-410m",
            "EleutherAI/pythia-410m-deduped": "pythia-410m", "EleutherAI/pythia-1.4b-deduped": "pythia-1.4b",
            "pythia-1.4b-deduped": "pythia-1.4b", "gpt2-small": "gpt2", "EleutherAI/pythia-160m": "pythia-160m"}
LAYER_LOCS = ("residual", "mlp", "attn", "mlpout")


def canonical_model_name(name: str) -> str:
    key = _ALIASES.get(name, name)
    if key not in MODEL_CONFIGS:
        raise ValueError(f"Model {name} not supported (known: {sorted(MODEL_CONFIGS)})")
    return key


def check_transformerlens_model(model_name: str) -> bool:
    """Reference API name; True for every architecture this harvester can build."""
    try:
        canonical_model_name(model_name)
        return True
    except ValueError:
        return False


def _dims(model_name: str) -> Dict[str, int]:
    c = MODEL_CONFIGS[canonical_model_name(model_name)]
    if c["arch"] == "gpt_neox":
        return dict(d_model=c["hidden_size"], d_mlp=c["intermediate_size"], n_heads=c["num_attention_heads"],
                    d_head=c["hidden_size"] // c["num_attention_heads"], n_layers=c["num_hidden_layers"],
                    vocab=c["vocab_size"])
    return dict(d_model=c["n_embd"], d_mlp=4 * c["n_embd"], n_heads=c["n_head"], d_head=c["n_embd"] // c["n_head"],
                n_layers=c["n_layer"], vocab=c["vocab_size"])


def get_activation_size(model_name: str, layer_loc: str) -> int:
    if layer_loc not in LAYER_LOCS:
        raise ValueError(f"Layer location {layer_loc} not supported")
    d = _dims(model_name)
    return {"residual": d["d_model"], "mlp": d["d_mlp"], "attn": d["d_head"] * d["n_heads"],
            "mlpout": d["d_model"]}[layer_loc]


def make_tensor_name(layer: int, layer_loc: str, model_name: str) -> str:
    """TransformerLens-style hook names (reference activation_dataset.py:78-109; attn fixed, B#13)."""
    check = canonical_model_name(model_name)  # noqa: F841 - validates the name
    return {"residual": f"blocks.{layer}.hook_resid_post", "mlp": f"blocks.{layer}.mlp.hook_post",
            "attn": f"blocks.{layer}.attn.hook_z", "mlpout": f"blocks.{layer}.hook_mlp_out"}[layer_loc]


def build_model(model_name: str, device="cuda", dtype=torch.bfloat16, seed: int = 0, pretrained_dir: str = ""):
    """Random-init (or local-checkpoint) HF model of the named architecture, eval mode."""
    import transformers

    key = canonical_model_name(model_name)
    c = dict(MODEL_CONFIGS[key])
    arch = c.pop("arch")
    torch.manual_seed(seed)
    if pretrained_dir and os.path.isdir(pretrained_dir):
        model = transformers.AutoModelForCausalLM.from_pretrained(pretrained_dir, torch_dtype=dtype)
    elif arch == "gpt_neox":
        cfg = transformers.GPTNeoXConfig(**c, use_parallel_residual=True, hidden_act="gelu")
        model = transformers.GPTNeoXForCausalLM(cfg)
    else:
        cfg = transformers.GPT2Config(**c)
        model = transformers.GPT2LMHeadModel(cfg)
    model = model.to(device=device, dtype=dtype).eval()
    model.requires_grad_(False)
    return model


class _Stop(Exception):
    pass


def _blocks(model):
    if hasattr(model, "gpt_neox"):
        return model.gpt_neox.layers, "gpt_neox"
    return model.transformer.h, "gpt2"


def _hook_module(model, layer: int, layer_loc: str):
    """(module, capture_input?) whose forward input/output is the requested activation."""
    blocks, arch = _blocks(model)
    blk = blocks[layer]
    if layer_loc == "residual":
        return blk, False
    if arch == "gpt_neox":
        if layer_loc == "mlp":
            return blk.mlp.dense_4h_to_h, True      # post-GELU hidden = input of the down projection
        if layer_loc == "mlpout":
            return blk.mlp, False
        return blk.attention.dense, True            # concatenated heads = input of the output projection
    if layer_loc == "mlp":
        return blk.mlp.c_proj, True
    if layer_loc == "mlpout":
        return blk.mlp, False
    return blk.attn.c_proj, True


class ActivationHarvester:
    """Runs token batches through a model and yields flattened ``[(b s), d]`` activations for
    one or more (layer, layer_loc) hook points."""

    def __init__(self, model, layers: Sequence[int], layer_loc: str = "residual", out_dtype=torch.bfloat16):
        self.model = model
        self.layers = list(layers)
        self.layer_loc = layer_loc
        self.out_dtype = out_dtype
        self._captured: Dict[int, torch.Tensor] = {}
        self._handles = []
        last = max(self.layers)
        for L in self.layers:
            mod, use_input = _hook_module(model, L, layer_loc)
            self._handles.append(mod.register_forward_hook(self._make_hook(L, use_input, L == last)))

    def _make_hook(self, layer, use_input, stop_after):
        def hook(mod, inputs, output):
            t = inputs[0] if use_input else (output[0] if isinstance(output, tuple) else output)
            self._captured[layer] = t.reshape(-1, t.shape[-1]).to(self.out_dtype)
            if stop_after and all(L in self._captured for L in self.layers):
                raise _Stop()  # stop_at_layer: skip the rest of the forward

        return hook

    @torch.no_grad()
    def run(self, tokens: torch.Tensor) -> Dict[int, torch.Tensor]:
        self._captured = {}
        try:
            self.model(input_ids=tokens)
        except _Stop:
            pass
        return dict(self._captured)

    def close(self):
        for h in self._handles:
            h.remove()
        self._handles = []


def synthetic_token_batches(vocab: int, batch: int = 32, seq_len: int = MAX_SENTENCE_LEN, seed: int = 0,
                            device="cpu", zipf_a: float = 1.1) -> Iterator[torch.Tensor]:
    """Endless Zipf-distributed token-id batches (offline stand-in for OpenWebText/Pile)."""
    g = torch.Generator().manual_seed(seed)
    ranks = torch.arange(1, vocab + 1, dtype=torch.float64)
    probs = (1.0 / ranks ** zipf_a)
    probs = (probs / probs.sum()).float()
    while True:
        yield torch.multinomial(probs, batch * seq_len, replacement=True, generator=g).view(batch, seq_len).to(device)


def chunk_and_tokenize(texts: Iterable[str], tokenizer, max_length: int = MAX_SENTENCE_LEN) -> torch.Tensor:
    """Concatenate texts with EOS separators and cut into ``max_length`` token rows
    (reference activation_dataset.py:139-238, without the HF-datasets dependency)."""
    eos = getattr(tokenizer, "eos_token_id", None)
    ids: List[int] = []
    for t in texts:
        ids.extend(tokenizer.encode(t))
        if eos is not None:
            ids.append(eos)
    n = len(ids) // max_length
    return torch.tensor(ids[: n * max_length], dtype=torch.long).view(n, max_length)


def harvest_to_ring(harvester: ActivationHarvester, token_batches: Iterator[torch.Tensor], rings: Dict[int, "object"],
                    n_rows: int, device="cuda", center: bool = False) -> Dict[int, Optional[torch.Tensor]]:
    """Fill one device ring per layer with ``n_rows`` activations; returns per-layer means
    (first-chunk mean, reference :308-311) when ``center``."""
    done = 0
    means: Dict[int, Optional[torch.Tensor]] = {L: None for L in rings}
    while done < n_rows:
        toks = next(token_batches).to(device)
        acts = harvester.run(toks)
        take = min(n_rows - done, next(iter(acts.values())).shape[0])
        for L, ring in rings.items():
            a = acts[L][:take]
            if center:
                if means[L] is None:
                    means[L] = a.float().mean(0)
                a = (a.float() - means[L]).to(a.dtype)
            ring.push(a)
        done += take
    return means


def setup_data(model_name: str = "pythia-70m", dataset_folder="activation_data", layer=2, layer_loc="residual",
               n_chunks: int = 1, chunk_size_gb: float = CHUNK_SIZE_GB, device="cuda", center_dataset=False,
               skip_chunks: int = 0, batch_size: int = MODEL_BATCH_SIZE * 16, seq_len: int = MAX_SENTENCE_LEN,
               token_batches: Optional[Iterator[torch.Tensor]] = None, seed: int = 0, model=None,
               rows_per_chunk: Optional[int] = None) -> int:
    """Write ``n_chunks`` reference-format chunks per layer (reference :400-460).

    ``dataset_folder``/``layer`` may be lists (several layers per forward, reference
    :326-391); returns the number of rows written per layer.
    """
    from .chunks import save_chunk

    layers = layer if isinstance(layer, (list, tuple)) else [layer]
    folders = dataset_folder if isinstance(dataset_folder, (list, tuple)) else [dataset_folder]
    assert len(layers) == len(folders)
    model = model or build_model(model_name, device=device, seed=seed)
    d = get_activation_size(model_name, layer_loc)
    rows = rows_per_chunk or int(chunk_size_gb * (1024 ** 3) // (d * 2))
    harv = ActivationHarvester(model, layers, layer_loc, out_dtype=torch.float16)
    toks = token_batches or synthetic_token_batches(_dims(model_name)["vocab"], batch_size, seq_len, seed=seed)
    means = {L: None for L in layers}
    written = 0
    try:
        for ci in range(skip_chunks + n_chunks):
            bufs = {L: [] for L in layers}
            have = 0
            while have < rows:
                acts = harv.run(next(toks).to(device))
                for L in layers:
                    bufs[L].append(acts[L])
                have += next(iter(acts.values())).shape[0]
            if ci < skip_chunks:
                continue
            for L, folder in zip(layers, folders):
                chunk = torch.cat(bufs[L])[:rows]
                if center_dataset:
                    if means[L] is None:
                        means[L] = chunk.float().mean(0)
                    chunk = (chunk.float() - means[L]).half()
                save_chunk(chunk, folder, ci - skip_chunks)
            written += rows
    finally:
        harv.close()
    return written
