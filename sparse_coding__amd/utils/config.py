"""Typed dataclass configs with explicit CLI parsing and YAML I/O.

Same field catalogue as reference ``config.py:29-140`` (``TrainArgs``,
``EnsembleArgs``, ``SyntheticEnsembleArgs``, ``ErasureArgs``, ``ToyArgs``,
``InterpArgs``, ``InterpGraphArgs``, ``InvestigateArgs``), fixing B#14/B#15:
constructing a config never reads ``sys.argv`` (call ``Cls.from_cli()``),
bools parse "false"/"0"/"no" correctly, ``torch.dtype`` fields parse
("float32", "bfloat16", ...), and the fields ``sweep`` uses
(``n_repetitions``, ``center_activations``) exist.
"""

from __future__ import annotations

import argparse
import dataclasses
import sys
from dataclasses import dataclass, field, fields
from typing import Any, Dict, List, Optional, Sequence

import torch
import yaml

_DTYPES = {"float32": torch.float32, "fp32": torch.float32, "float16": torch.float16, "fp16": torch.float16,
           "bfloat16": torch.bfloat16, "bf16": torch.bfloat16, "float64": torch.float64}


def parse_bool(s: str) -> bool:
    v = str(s).strip().lower()
    if v in ("1", "true", "yes", "y", "on"):
        return True
    if v in ("0", "false", "no", "n", "off"):
        return False
    raise argparse.ArgumentTypeError(f"not a boolean: {s!r}")


def parse_dtype(s) -> torch.dtype:
    if isinstance(s, torch.dtype):
        return s
    key = str(s).replace("torch.", "")
    if key not in _DTYPES:
        raise argparse.ArgumentTypeError(f"unknown dtype {s!r}")
    return _DTYPES[key]


def _parser_for(default):
    if isinstance(default, bool):
        return parse_bool
    if isinstance(default, torch.dtype):
        return parse_dtype
    if isinstance(default, int):
        return int
    if isinstance(default, float):
        return float
    if isinstance(default, (list, tuple)):
        return lambda s: [type(default[0])(x) if default else x for x in s.split(",")]
    return str


@dataclass
class BaseArgs:
    """Base config: ``Cls.from_cli(argv)`` builds an instance and applies ``--field value`` flags."""

    @classmethod
    def arg_parser(cls) -> argparse.ArgumentParser:
        p = argparse.ArgumentParser(description=cls.__doc__)
        inst = cls()
        for f in fields(cls):
            default = getattr(inst, f.name)
            typ = _parser_for(default) if default is not None else str
            p.add_argument(f"--{f.name}", type=typ, default=None, help=f"(default: {default!r})")
        p.add_argument("--config", type=str, default=None, help="YAML file with field values")
        return p

    @classmethod
    def from_cli(cls, argv: Optional[Sequence[str]] = None):
        ns = cls.arg_parser().parse_args(sys.argv[1:] if argv is None else list(argv))
        inst = cls.from_yaml(ns.config) if ns.config else cls()
        for f in fields(cls):
            v = getattr(ns, f.name)
            if v is not None:
                setattr(inst, f.name, v)
        return inst

    def update(self, values: Dict[str, Any]):
        names = {f.name for f in fields(self)}
        unknown = set(values) - names
        if unknown:
            raise ValueError(f"Unknown arguments: {sorted(unknown)}")
        for k, v in values.items():
            if v is not None:
                setattr(self, k, v)
        return self

    def to_dict(self) -> Dict[str, Any]:
        out = {}
        for f in fields(self):
            v = getattr(self, f.name)
            out[f.name] = str(v).replace("torch.", "") if isinstance(v, torch.dtype) else v
        return out

    def to_yaml(self, path: str):
        with open(path, "w") as fh:
            yaml.safe_dump(self.to_dict(), fh, sort_keys=True)

    @classmethod
    def from_yaml(cls, path: str):
        with open(path) as fh:
            data = yaml.safe_load(fh) or {}
        inst = cls()
        for f in fields(cls):
            if f.name in data:
                v = data[f.name]
                if isinstance(getattr(inst, f.name), torch.dtype):
                    v = parse_dtype(v)
                setattr(inst, f.name, v)
        return inst

    # reference code calls dict(cfg) (B#14): support it
    def keys(self):
        return [f.name for f in fields(self)]

    def __getitem__(self, k):
        return getattr(self, k)


def _default_device() -> str:
    return "cuda:0" if torch.cuda.is_available() else "cpu"


@dataclass
class TrainArgs(BaseArgs):
    """Training defaults of record (reference config.py:29-52)."""

    layer: int = 2
    layer_loc: str = "residual"
    model_name: str = "pythia-70m-deduped"
    dataset_name: str = "openwebtext"
    dataset_folder: str = ""
    device: str = field(default_factory=_default_device)
    tied_ae: bool = False
    seed: int = 0
    learned_dict_ratio: float = 1.0
    output_folder: str = "outputs"
    dtype: torch.dtype = torch.float32
    epochs: int = 1
    center_dataset: bool = False
    n_chunks: int = 30
    chunk_size_gb: float = 2.0
    batch_size: int = 256
    use_wandb: bool = False
    wandb_images: bool = False
    lr: float = 1e-3
    l1_alpha: float = 1e-3
    save_every: int = 5
    n_epochs: int = 1
    # fields the reference's sweep() reads but never declared (B#14)
    n_repetitions: int = 1
    center_activations: bool = False
    # MI355X engine knobs
    engine: str = "auto"            # auto | fused | eager
    use_graph: bool = True
    log_every: int = 100
    log_dir: str = ""
    resume: bool = True


@dataclass
class EnsembleArgs(TrainArgs):
    activation_width: int = 512
    use_synthetic_dataset: bool = False
    bias_decay: float = 0.0


@dataclass
class SyntheticEnsembleArgs(EnsembleArgs):
    noise_magnitude_scale: float = 0.0
    feature_prob_decay: float = 0.99
    feature_num_nonzero: int = 10
    gen_batch_size: int = 4096
    dataset_folder: str = "activation_data"
    n_ground_truth_components: int = 512
    correlated_components: bool = False


@dataclass
class ErasureArgs(BaseArgs):
    model_name: str = "EleutherAI/pythia-70m-deduped"
    device: str = field(default_factory=_default_device)
    layer: int = -1
    count_cutoff: int = 10000
    output_folder: str = "output_erasure_pca"
    activation_filename: str = "activation_data_erasure.pt"
    dict_filename: str = ""


@dataclass
class ToyArgs(BaseArgs):
    layer: int = 2
    layer_loc: str = "residual"
    model_name: str = "pythia-70m-deduped"
    dataset_name: str = "openwebtext"
    device: str = field(default_factory=_default_device)
    tied_ae: bool = False
    seed: int = 0
    learned_dict_ratio: float = 1.0
    output_folder: str = "outputs"
    dtype: torch.dtype = torch.float32
    activation_dim: int = 256
    feature_prob_decay: float = 0.99
    feature_num_nonzero: int = 5
    correlated_components: bool = False
    n_ground_truth_components: int = 512
    noise_std: float = 0.1
    l1_exp_low: int = -12
    l1_exp_high: int = -11
    l1_exp_base: float = 10 ** (1 / 4)
    dict_ratio_exp_low: int = 1
    dict_ratio_exp_high: int = 7
    dict_ratio_exp_base: float = 2.0
    batch_size: int = 4096
    lr: float = 1e-3
    epochs: int = 1
    noise_level: float = 0.0
    n_components_dictionary: int = 512
    l1_alpha: float = 1e-3


@dataclass
class InterpArgs(BaseArgs):
    layer: int = 2
    model_name: str = "EleutherAI/pythia-70m-deduped"
    layer_loc: str = "residual"
    device: str = field(default_factory=_default_device)
    n_feats_explain: int = 10
    load_interpret_autoencoder: str = ""
    tied_ae: bool = False
    interp_name: str = ""
    sort_mode: str = "max"
    use_decoder: bool = True
    df_n_feats: int = 200
    top_k: int = 50
    save_loc: str = ""
    # MI355X / offline additions
    n_fragments: int = 50000
    fragment_len: int = 64
    batch_size: int = 256
    token_file: str = ""              # LongTensor [N, S] of documents; synthetic Zipf stream if empty
    explainer: str = "offline"        # offline | endpoint (SC_INTERP_ENDPOINT)
    explainer_model: str = "gpt-4"
    simulator_model: str = "gpt-3.5-turbo"
    seed: int = 0


@dataclass
class InterpGraphArgs(BaseArgs):
    layer: int = 1
    model_name: str = "EleutherAI/pythia-70m-deduped"
    layer_loc: str = "mlp"
    score_mode: str = "all"
    run_all: bool = False


@dataclass
class InvestigateArgs(BaseArgs):
    threshold: float = 0.9
    layer: int = 2
    device: str = field(default_factory=_default_device)


@dataclass
class SweepArgs(EnsembleArgs):
    """The fork's FISTA sweep CLI (reference basic_l1_sweep.py:126-136)."""

    dataset_dir: str = "activation_data/layer_2"
    output_dir: str = "output_basic_test/fista_sweep"
    l1_value_min: float = -4.0
    l1_value_max: float = -2.0
    l1_value_n: int = 4
    ratio: float = 1.0
    save_after_every: bool = True
    adam_lr: float = 1e-3
    fista_iters: int = 500
    fista_backend: str = "auto"
    fista_eta: str = "tracked"        # "eigh" reproduces the reference's exact eigvalsh per call
    persist_hessian: bool = False     # reference quirk B#3 (throwaway EMA) by default
    basis_normalize: str = "column"   # reference quirk B#4 by default
    signature: str = "fista"          # fista | fista_loss | sae | tied
    parallel: str = "none"            # "es": ensemble-axis sharding over torchrun ranks


def make_hyperparam_name(values: Dict[str, Any]) -> str:
    """``{"l1_alpha": 1e-3}`` -> ``"l1_alpha_1.00E-03"`` (reference big_sweep.py:76-84)."""
    parts = []
    for k, v in values.items():
        parts.append(f"{k}_{v:.2E}" if isinstance(v, float) else f"{k}_{v}")
    return "_".join(parts)
