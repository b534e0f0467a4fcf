"""Experiment catalogue: ensemble-init functions and ``run_*`` entry points.

Same sweeps as reference ``big_sweep_experiments.py:40-1286``; each init function
returns ``(ensembles, ensemble_hparams, buffer_hparams, hparam_ranges)`` with
``ensembles`` a list of ``(models, sig, args, name)``.  Device placement is not
hard-coded (the reference pins ensembles to ``cuda:0..7``): ``sweep`` shards
ensembles over the ranks of the job.

CLI:  ``python -m sparse_coding__amd.train.experiments <run_name> [--field value ...]``
"""

from __future__ import annotations

import sys
from itertools import product
from typing import Callable, Dict, List, Tuple

import numpy as np

from ..models.fista import FunctionalFista
from ..models.lista import FunctionalLISTADenoisingSAE
from ..models.misc import FunctionalPositiveTiedSAE
from ..models.signatures import (FunctionalMaskedTiedSAE, FunctionalSAE, FunctionalThresholdingSAE,
                                 FunctionalTiedSAE)
from ..models.topk import TopKEncoder
from ..utils.config import EnsembleArgs, SyntheticEnsembleArgs


def _args(cfg, dict_size, **extra):
    out = {"batch_size": cfg.batch_size, "device": cfg.device, "dict_size": dict_size}
    out.update(extra)
    return out


def _sae(cfg):
    return FunctionalTiedSAE if cfg.tied_ae else FunctionalSAE


# ----------------------------------------------------------------------------- init functions
def tied_vs_not_experiment(cfg):
    """Untied vs tied at ratio 8 over an L1 x bias-decay grid (reference :40-230)."""
    l1_values = list(np.logspace(-3.5, -2, 4))
    bias_decays = [0.0, 0.05, 0.1]
    n = cfg.activation_width * 8
    ensembles = []
    for tied in (False, True):
        sig = FunctionalTiedSAE if tied else FunctionalSAE
        for i in range(2):
            grid = list(product(l1_values[i * 2:(i + 1) * 2], bias_decays))
            models = [sig.init(cfg.activation_width, n, float(l1), bias_decay=bd) for l1, bd in grid]
            name = f"dict_ratio_8_group_{i}" + ("_tied" if tied else "")
            ensembles.append((models, sig, _args(cfg, n, tied=tied), name))
    return ensembles, ["tied", "dict_size"], ["l1_alpha", "bias_decay"], \
        {"tied": [False, True], "dict_size": [n], "l1_alpha": l1_values, "bias_decay": bias_decays}


def topk_experiment(cfg):
    """Top-k sweep: k in 1..151 step 10 for 8 dictionary ratios (reference :233-263)."""
    sparsity = np.arange(1, 161, 10)
    ratios = [0.5, 1, 2, 4, 0.5, 1, 2, 4]
    ensembles = []
    for i, r in enumerate(ratios):
        n = int(cfg.activation_width * r)
        models = [TopKEncoder.init(cfg.activation_width, n, int(min(k, n))) for k in sparsity]
        ensembles.append((models, TopKEncoder, _args(cfg, n), f"topk_{i}"))
    return ensembles, ["dict_size"], ["sparsity"], \
        {"dict_size": [int(cfg.activation_width * r) for r in ratios], "sparsity": sparsity}


def synthetic_linear_range(cfg):
    l1_vals = np.logspace(-4, -2, 32)
    ratios = [0.5, 1, 2, 4]
    settings = list(product([l1_vals[:16], l1_vals[16:]], ratios))
    ensembles = []
    for i, (l1_range, r) in enumerate(settings):
        n = int(cfg.activation_width * r)
        models = [FunctionalTiedSAE.init(cfg.activation_width, n, float(l1)) for l1 in l1_range]
        ensembles.append((models, FunctionalTiedSAE, _args(cfg, n), f"synthetic_{i}"))
    return ensembles, ["dict_size"], ["l1_alpha"], \
        {"dict_size": [int(cfg.activation_width * r) for r in ratios], "l1_alpha": l1_vals}


def dense_l1_range_experiment(cfg):
    l1_values = np.logspace(-4, -2, 16)
    n = int(cfg.activation_width * cfg.learned_dict_ratio)
    sig = _sae(cfg)
    ensembles = [([sig.init(cfg.activation_width, n, float(l1), bias_decay=0.0)], sig, _args(cfg, n),
                  f"l1_range_8_{i}") for i, l1 in enumerate(l1_values[:8])]
    return ensembles, ["dict_size"], ["l1_alpha"], {"dict_size": [n], "l1_alpha": l1_values}


def residual_denoising_experiment(cfg):
    l1_values = np.logspace(-5, -3, 16)
    n = int(cfg.activation_width * cfg.learned_dict_ratio)
    ensembles = []
    for i in range(4):
        models = [FunctionalLISTADenoisingSAE.init(cfg.activation_width, n, 3, float(l1))
                  for l1 in l1_values[i * 4:(i + 1) * 4]]
        ensembles.append((models, FunctionalLISTADenoisingSAE, _args(cfg, n), f"residual_denoising_{i}"))
    return ensembles, ["dict_size"], ["l1_alpha"], {"dict_size": [n], "l1_alpha": l1_values}


def residual_denoising_comparison(cfg):
    l1_values = np.logspace(-4, -2, 16)
    n = int(cfg.activation_width * cfg.learned_dict_ratio)
    ensembles = [([FunctionalTiedSAE.init(cfg.activation_width, n, float(l1)) for l1 in l1_values[i * 4:(i + 1) * 4]],
                  FunctionalTiedSAE, _args(cfg, n), f"residual_denoising_cmp_{i}") for i in range(4)]
    return ensembles, ["dict_size"], ["l1_alpha"], {"dict_size": [n], "l1_alpha": l1_values}


def thresholding_experiment(cfg):
    l1_values = np.logspace(-4, -2, 16)
    n = int(cfg.activation_width * 4)
    ensembles = [([FunctionalThresholdingSAE.init(cfg.activation_width, n, float(l1))
                   for l1 in l1_values[i * 4:(i + 1) * 4]], FunctionalThresholdingSAE, _args(cfg, n),
                  f"thresholding_{i}") for i in range(4)]
    return ensembles, ["dict_size"], ["l1_alpha"], {"dict_size": [n], "l1_alpha": l1_values}


def zero_l1_baseline(cfg):
    n = int(cfg.activation_width * 4)
    sig = _sae(cfg)
    return [([sig.init(cfg.activation_width, n, 0.0, bias_decay=0.0)], sig, _args(cfg, n), "l1_range_zero_b")], \
        ["dict_size"], ["l1_alpha"], {"dict_size": [n], "l1_alpha": [0.0]}


def dict_ratio_experiment(cfg):
    """Masked tied SAEs of 8 sizes x 12 repeats stacked into one ensemble (reference :546-580)."""
    sizes = [int(512 * x) for x in np.linspace(1, 5, 8)]
    stack = max(sizes)
    stack = ((stack + 127) // 128) * 128  # pad the stack to the kernel tile
    ensembles = []
    for i in range(6):
        models = [FunctionalMaskedTiedSAE.init(cfg.activation_width, s, stack, 1e-3) for _ in range(12) for s in sizes]
        ensembles.append((models, FunctionalMaskedTiedSAE, _args(cfg, stack), f"l1_{i}"))
    return ensembles, [], ["l1_alpha", "dict_size"], {"dict_size": sizes, "l1_alpha": [1e-3]}


def pythia_1_4_b_dict(cfg):
    n = int(cfg.activation_width * 6)
    l1_values = np.logspace(-4, -2, 5)
    return [([FunctionalTiedSAE.init(cfg.activation_width, n, float(l1)) for l1 in l1_values], FunctionalTiedSAE,
             _args(cfg, n), "l1_0")], [], ["l1_alpha"], {"dict_size": [n], "l1_alpha": l1_values}


def run_zeros_only_init(cfg):
    n = int(cfg.activation_width * cfg.learned_dict_ratio)
    sig = _sae(cfg)
    return [([sig.init(cfg.activation_width, n, 0.0)], sig, _args(cfg, n), f"l1_range_zero")], \
        ["dict_size"], ["l1_alpha"], {"dict_size": [n], "l1_alpha": [0.0]}


def long_mlp_sweep(cfg):
    l1_values = np.concatenate([[0.0, 1e-4], np.logspace(-3.5, -2.5, 5)])
    n = int(cfg.activation_width * cfg.learned_dict_ratio)
    sig = _sae(cfg)
    return [([sig.init(cfg.activation_width, n, float(l1)) for l1 in l1_values], sig, _args(cfg, n), "long_mlp")], \
        ["dict_size"], ["l1_alpha"], {"dict_size": [n], "l1_alpha": l1_values}


def run_positive_init(cfg):
    l1_values = np.concatenate([[0.0], np.logspace(-5, -3.5, 8)])
    n = int(cfg.activation_width * cfg.learned_dict_ratio)
    return [([FunctionalPositiveTiedSAE.init(cfg.activation_width, n, float(l1)) for l1 in l1_values],
             FunctionalPositiveTiedSAE, _args(cfg, n), "positive")], ["dict_size"], ["l1_alpha"], \
        {"dict_size": [n], "l1_alpha": l1_values}


def simple_setoff(cfg):
    """L1 in {0} u logspace(-4, -2, 8), one ensemble (reference :1099-1143)."""
    l1_values = np.concatenate([[0.0], np.logspace(-4, -2, 8)])
    n = int(cfg.activation_width * cfg.learned_dict_ratio)
    sig = _sae(cfg)
    models = [sig.init(cfg.activation_width, n, float(l1), bias_decay=0.0) for l1 in l1_values]
    return [(models, sig, _args(cfg, n), f"simple_{cfg.device}")], ["dict_size"], ["l1_alpha"], \
        {"dict_size": [n], "l1_alpha": l1_values}


def fista_sweep(cfg):
    """The fork's FISTA dictionary-learning sweep as an init function."""
    l1_values = np.logspace(getattr(cfg, "l1_value_min", -4), getattr(cfg, "l1_value_max", -2),
                            getattr(cfg, "l1_value_n", 4))
    n = int(cfg.activation_width * getattr(cfg, "ratio", cfg.learned_dict_ratio))
    models = [FunctionalFista.init(cfg.activation_width, n, float(l1)) for l1 in l1_values]
    return [(models, FunctionalFista, _args(cfg, n), "fista")], ["dict_size"], ["l1_alpha"], \
        {"dict_size": [n], "l1_alpha": l1_values}


def fista_in_loss_sweep(cfg):
    """The fork's "FISTA in the loss" runs (fista_13_10, output_basic_test/filename_explanations.txt:7-8;
    reference autoencoders/fista.py:141-172): tied normalised SAE + the residual of 50 unrolled
    FISTA iterations warm-started from the codes, over an L1 sweep."""
    l1_values = np.logspace(getattr(cfg, "l1_value_min", -4), getattr(cfg, "l1_value_max", -2),
                            getattr(cfg, "l1_value_n", 4))
    n = int(cfg.activation_width * getattr(cfg, "ratio", cfg.learned_dict_ratio))
    models = [FunctionalFista.init(cfg.activation_width, n, float(l1)) for l1 in l1_values]
    args = dict(_args(cfg, n), objective="fista_loss", fista_loss_iters=int(getattr(cfg, "fista_loss_iters", 50)))
    return [(models, FunctionalFista, args, "fista_loss")], ["dict_size"], ["l1_alpha"], \
        {"dict_size": [n], "l1_alpha": l1_values}


INIT_FUNCS: Dict[str, Callable] = {f.__name__: f for f in [
    fista_in_loss_sweep, tied_vs_not_experiment, topk_experiment, synthetic_linear_range, dense_l1_range_experiment,
    residual_denoising_experiment, residual_denoising_comparison, thresholding_experiment, zero_l1_baseline,
    dict_ratio_experiment, pythia_1_4_b_dict, run_zeros_only_init, long_mlp_sweep, run_positive_init,
    simple_setoff, fista_sweep]}


# ----------------------------------------------------------------------------- run_* entry points
def _cfg(argv, cls=EnsembleArgs, **overrides):
    """Experiment defaults, then ``--field value`` flags from ``argv`` on top."""
    cfg = cls().update(overrides)
    if argv:
        ns = cls.arg_parser().parse_args(list(argv))
        cfg.update({k: v for k, v in vars(ns).items() if v is not None and k != "config"})
    return cfg


def run_single_layer(argv=None):
    """Pythia-70m residual, tied, ratios 4..32, centred (reference :1211-1242)."""
    from .sweep import sweep

    base = dict(model_name="pythia-70m-deduped", batch_size=1024, tied_ae=True, center_dataset=True, n_epochs=5,
                n_chunks=16, lr=1e-3, layer_loc="residual")
    for ratio in (4, 8, 16, 32):
        cfg = _cfg(argv, **base, learned_dict_ratio=float(ratio),
                   dataset_folder="activation_data/pythia70m_resid_l2",
                   output_folder=f"outputs/pythia70m_tied_resid_r{ratio}")
        sweep(simple_setoff, cfg)


def run_single_layer_gpt2(argv=None):
    from .sweep import sweep

    for ratio in (32, 64, 96):
        cfg = _cfg(argv, model_name="gpt2", batch_size=1024, tied_ae=True, learned_dict_ratio=float(ratio),
                   dataset_folder="activation_data/gpt2_resid_l2", output_folder=f"outputs/gpt2_tied_resid_r{ratio}")
        sweep(simple_setoff, cfg)


def run_across_layers_mlp_long(argv=None):
    from .sweep import sweep

    for tied in (True, False):
        for ratio in (0.25, 0.5, 1.0, 2.0, 4.0, 8.0, 16.0):
            cfg = _cfg(argv, model_name="pythia-70m-deduped", batch_size=2048, layer_loc="mlp", tied_ae=tied,
                       learned_dict_ratio=ratio, dataset_folder="activation_data/pythia70m_mlp",
                       output_folder=f"outputs/{'tied' if tied else 'untied'}_mlp_r{ratio}_long")
            sweep(long_mlp_sweep, cfg)


def run_pythia_1_4_b_sweep(argv=None):
    from .sweep import sweep

    cfg = _cfg(argv, model_name="pythia-1.4b", batch_size=1024, n_chunks=30, n_epochs=10, layer=6,
               dataset_folder="activation_data_1_4_b", output_folder="output_1_4_b")
    sweep(pythia_1_4_b_dict, cfg)


def run_synthetic(argv=None):
    from .sweep import sweep

    cfg = _cfg(argv, cls=SyntheticEnsembleArgs, use_synthetic_dataset=True, n_chunks=4, chunk_size_gb=0.25,
               dataset_folder="activation_data/synthetic", output_folder="outputs/synthetic")
    sweep(synthetic_linear_range, cfg)


def _synthetic_base(argv, **overrides):
    """The reference's synthetic-shape defaults for its real-data runs (activation width 512,
    1024 ground-truth features, 10 nonzero, decay 0.99, noise 1e-3)."""
    base = dict(model_name="pythia-70m-deduped", layer=2, layer_loc="residual", n_chunks=10, batch_size=1024,
                gen_batch_size=4096, n_ground_truth_components=1024, activation_width=512,
                noise_magnitude_scale=0.001, feature_prob_decay=0.99, feature_num_nonzero=10, lr=1e-3)
    base.update(overrides)
    return _cfg(argv, cls=SyntheticEnsembleArgs, **base)


def run_thresholding(argv=None):
    """Thresholding SAEs on Pythia-70m layer-2 residual chunks (reference :437-464)."""
    from .sweep import sweep

    sweep(thresholding_experiment, _synthetic_base(argv, dataset_folder="activation_data",
                                                   output_folder="output_thresholding"))


def run_resid_denoise(argv=None):
    """LISTA residual-denoising SAEs at dict ratio 4 (reference :467-496)."""
    from .sweep import sweep

    for ratio in (4,):
        sweep(residual_denoising_experiment, _synthetic_base(argv, dataset_folder="activation_data",
                                                             learned_dict_ratio=float(ratio),
                                                             output_folder=f"output_{ratio}_lista_neg"))


def run_dict_ratio(argv=None):
    """Masked tied SAEs of 8 dictionary sizes stacked in one ensemble, synthetic data
    (reference :583-620)."""
    from .sweep import sweep

    cfg = _cfg(argv, cls=SyntheticEnsembleArgs, model_name="pythia-70m-deduped", layer=4, layer_loc="residual",
               use_synthetic_dataset=True, lr=1e-3, n_chunks=10, correlated_components=False, chunk_size_gb=2.0,
               batch_size=1024, n_epochs=1, dataset_folder="activation_data", output_folder="output_dict_ratio")
    sweep(dict_ratio_experiment, cfg)


def run_dense_l1_range(argv=None):
    """Dense L1 range on Pythia-70m layer-3 MLP, tied (reference :623-643)."""
    from .sweep import sweep

    cfg = _cfg(argv, model_name="pythia-70m-deduped", batch_size=2048, layer_loc="mlp", layer=3, bias_decay=0.0,
               tied_ae=True, use_synthetic_dataset=False, lr=1e-3, n_chunks=20, n_epochs=15)
    if not cfg.output_folder or cfg.output_folder == "outputs":
        cfg.output_folder = f"normal_{'_tied' if cfg.tied_ae else ''}_{cfg.layer_loc}_l{cfg.layer}_r{int(cfg.learned_dict_ratio)}"
    if not cfg.dataset_folder:
        cfg.dataset_folder = f"pilechunks_l{cfg.layer}_{cfg.layer_loc}"
    sweep(dense_l1_range_experiment, cfg)


def _across_layers(argv, init, layers, locs, ratios, tied, lr, base_out, **extra):
    from .sweep import sweep

    for layer in layers:
        for loc in locs:
            for ratio in ratios:
                cfg = _cfg(argv, model_name="pythia-70m-deduped", tied_ae=tied, layer=layer, layer_loc=loc,
                           learned_dict_ratio=float(ratio), use_synthetic_dataset=False, lr=lr,
                           dataset_folder=f"pilechunks_l{layer}_{loc}",
                           output_folder=f"{base_out}{'_tied' if tied else ''}_{loc}_l{layer}_r{int(ratio)}", **extra)
                sweep(init, cfg)


def run_across_layers(argv=None):
    """Tied residual dictionaries (ratio 4) for layers 0-5 (reference :646-679)."""
    _across_layers(argv, simple_setoff, range(6), ["residual"], [4], True, 1e-3, "longrun",
                   batch_size=1024, save_every=5, n_chunks=20, n_epochs=20)


def run_across_layers_attn(argv=None):
    """Attention-output dictionaries, ratios 1-8, layers 0-5 (reference :682-710)."""
    _across_layers(argv, dense_l1_range_experiment, range(6), ["attn"], [1, 2, 4, 8], True, 3e-4,
                   "output_attn_sweep", batch_size=2048, save_every=2, n_chunks=10)


def run_across_layers_mlp_out(argv=None):
    """MLP-out (hook_mlp_out, d_model wide) dictionaries, ratios 1-8 (reference :713-741)."""
    _across_layers(argv, dense_l1_range_experiment, [0, 1, 3, 4, 5], ["mlpout"], [1, 2, 4, 8], True, 3e-4,
                   "output_sweep", batch_size=2048, save_every=2, n_chunks=10)


def run_across_layers_mlp_untied(argv=None):
    """Untied MLP (hook_post, d_mlp wide) dictionaries, ratios 1-8 (reference :744-772)."""
    _across_layers(argv, dense_l1_range_experiment, range(6), ["mlp"], [1, 2, 4, 8], False, 3e-4, "output_sweep",
                   batch_size=2048, save_every=2, n_chunks=10)


def run_zero_l1_baseline(argv=None):
    """L1 = 0 tied baseline on layer-3 residual, ratio 4 (reference :775-796)."""
    from .sweep import sweep

    cfg = _cfg(argv, model_name="pythia-70m-deduped", layer=3, layer_loc="residual", tied_ae=True,
               learned_dict_ratio=4.0, batch_size=2048, output_folder="output_zero_b_4",
               dataset_folder="activation_data/layer_3", use_synthetic_dataset=False, lr=3e-4, n_chunks=38)
    sweep(zero_l1_baseline, cfg)


def run_topk(argv=None):
    """Top-k encoder sweep (reference ``topk`` :799-814)."""
    from .sweep import sweep

    cfg = _cfg(argv, model_name="pythia-70m-deduped", batch_size=1024, output_folder="output_topk",
               dataset_folder="activation_data", use_synthetic_dataset=False, lr=1e-3, n_chunks=10, n_epochs=5)
    sweep(topk_experiment, cfg)


def run_fista_in_loss(argv=None):
    """FISTA-in-the-loss L1 sweep, dict_size = d (the fork's fista_13_10 runs; d = 512 on Pythia-70m)."""
    from .sweep import sweep

    cfg = _cfg(argv, model_name="pythia-70m-deduped", batch_size=1024, output_folder="output_fista_loss",
               dataset_folder="activation_data", use_synthetic_dataset=False, lr=1e-3, n_chunks=10,
               learned_dict_ratio=1.0)
    sweep(fista_in_loss_sweep, cfg)


def run_synthetic_test(argv=None):
    """Synthetic ground-truth grid: n_ground_truth in {1024, 2048} x nonzero in {10, 50, 100},
    noise 0.1 (reference ``synthetic_test`` :817-851)."""
    from .sweep import remove_synthetic_dataset, sweep

    for noise, nz, ngt in product([0.1], [10, 50, 100], [1024, 2048]):
        cfg = _cfg(argv, cls=SyntheticEnsembleArgs, use_synthetic_dataset=True,
                   dataset_folder="activation_data_synthetic", batch_size=1024, gen_batch_size=4096,
                   activation_width=512, feature_prob_decay=1.0, lr=1e-3, n_chunks=10, correlated_components=False,
                   noise_magnitude_scale=noise, n_ground_truth_components=ngt, feature_num_nonzero=nz,
                   output_folder=f"output_synthetic_{noise:.2E}_{ngt}_{nz}")
        remove_synthetic_dataset(cfg.dataset_folder)  # regenerate per setting (only our own generated chunks)
        sweep(synthetic_linear_range, cfg)


def run_setup_positives(argv=None):
    """Positive tied SAEs on the MLP (bias decay 0.01, ratio 1; reference ``setup_positives``
    :1071-1096)."""
    from .sweep import sweep

    for bias_decay in (0.01,):
        for ratio in (1.0,):
            cfg = _cfg(argv, model_name="pythia-70m-deduped", batch_size=2048, save_every=10, tied_ae=True,
                       use_synthetic_dataset=False, lr=1e-3, n_chunks=20, n_epochs=15, activation_width=2048,
                       layer_loc="mlp", bias_decay=bias_decay, learned_dict_ratio=ratio)
            cfg.output_folder = f"positive_{cfg.layer_loc}_l{cfg.layer}_r{cfg.learned_dict_ratio}_bd{cfg.bias_decay}"
            cfg.dataset_folder = f"pilechunks_l{cfg.layer}_{cfg.layer_loc}"
            sweep(run_positive_init, cfg)


def run_all_zeros(argv=None):
    """L1 = 0 dictionaries over tied/untied x {residual, mlpout} x ratios 0.5-32 for one layer
    (reference :1146-1177; ``--layer`` / ``--device`` from the command line)."""
    from .sweep import sweep

    for tied in (True, False):
        for loc in ("residual", "mlpout"):
            for ratio in (0.5, 1, 2, 4, 8, 16, 32):
                cfg = _cfg(argv, model_name="pythia-70m-deduped", batch_size=2048, save_every=10,
                           use_synthetic_dataset=False, lr=1e-3, activation_width=2048, tied_ae=tied, layer_loc=loc,
                           learned_dict_ratio=float(ratio), n_chunks=20 if loc == "mlp" else 10,
                           n_epochs=3 if loc == "mlp" else 1)
                cfg.output_folder = f"zeros_{loc}_l{cfg.layer}_r{cfg.learned_dict_ratio}_{'tied' if tied else 'untied'}"
                cfg.dataset_folder = f"pilechunks_l{cfg.layer}_{loc}"
                sweep(run_zeros_only_init, cfg)


def run_simple(argv=None):
    """GPT-2-small layer-6 MLP, untied, ratio 4 (reference ``simple_run`` :1180-1208)."""
    from datetime import datetime

    from .sweep import sweep

    cfg = _cfg(argv, model_name="gpt2", batch_size=2048, save_every=10, use_synthetic_dataset=False, lr=1e-3,
               n_chunks=40, n_epochs=10, activation_width=2048, layer=6, layer_loc="mlp", tied_ae=False,
               learned_dict_ratio=4.0)
    stamp = datetime.now().strftime("%Y-%m-%d_%H-%M-%S")
    cfg.output_folder = f"gpt2small_{'tied' if cfg.tied_ae else 'untied'}_{cfg.layer_loc}_l{cfg.layer}_r{cfg.learned_dict_ratio}_{stamp}"
    cfg.dataset_folder = f"pilechunks_l{cfg.layer}_{cfg.layer_loc}_gpt2"
    sweep(simple_setoff, cfg)


RUNS = {f.__name__: f for f in [run_single_layer, run_single_layer_gpt2, run_across_layers_mlp_long,
                                run_pythia_1_4_b_sweep, run_synthetic, run_thresholding, run_resid_denoise,
                                run_dict_ratio, run_dense_l1_range, run_across_layers, run_across_layers_attn,
                                run_across_layers_mlp_out, run_across_layers_mlp_untied, run_zero_l1_baseline,
                                run_topk, run_fista_in_loss, run_synthetic_test, run_setup_positives, run_all_zeros, run_simple]}


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] not in RUNS and argv[0] not in INIT_FUNCS:
        print("usage: python -m sparse_coding__amd.train.experiments <run|init_func> [--field value ...]")
        print("runs:", ", ".join(RUNS))
        print("init functions (with --dataset_folder/--output_folder):", ", ".join(INIT_FUNCS))
        return 2
    name, rest = argv[0], argv[1:]
    if name in RUNS:
        RUNS[name](rest)
    else:
        from .sweep import sweep

        sweep(INIT_FUNCS[name], EnsembleArgs.from_cli(rest))
    return 0


if __name__ == "__main__":
    sys.exit(main())
