"""Sweep orchestration: train many ensembles over activation chunks, checkpoint, resume.

Reference: ``big_sweep.py:161-429`` (``ensemble_train_loop``, ``sweep``,
``unstacked_to_learned_dicts``, checkpoint schedule) and ``cluster_runs.py``
(one process per ensemble per GPU over a shared CPU chunk).  MI355X design:

* each process drives one GPU (``torchrun`` style); its ensembles train back to
  back on the chunk held in that GPU's HBM ring -- no per-batch H2D copies;
* with several ranks the ensembles are *sweep-sharded* (ensemble i on rank
  i % world, reference P2) -- no gradient traffic -- and every rank reads the same
  chunk with the native prefetcher (next chunk streams from disk during training);
* checkpoints: reference-layout ``learned_dicts.pt`` + ``config.yaml`` at chunk
  counts 8, 16, ..., 512 and at the end (reference :421-427), plus a native
  resumable state (params + Adam + step + RNG + chunk cursor) after every chunk.

The ensemble-init contract is the reference's (``big_sweep_experiments.py:32-36``):
``init_func(cfg) -> (list[(models, sig, args, name)], ensemble_hparams,
buffer_hparams, hparam_ranges)`` where ``models`` is the list of per-model
``(params, buffers)`` that ``FunctionalEnsemble`` would stack.
"""

from __future__ import annotations

import datetime
import os
import time
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..data.chunks import ChunkFolder
from ..data.ring import DeviceRing
from ..engine.trainer import EnsembleTrainer
from ..parallel.dist import DistInfo, barrier, init_distributed
from ..utils import checkpoint as ckpt
from ..utils.config import make_hyperparam_name
from ..utils.logging import Logger, model_metric_names, trace_range

CHECKPOINT_COUNTS = [2 ** j for j in range(3, 10)]


def ensemble_train_loop(trainer: EnsembleTrainer, ring: DeviceRing, batch_size: int, n_batches: Optional[int] = None,
                        logger: Optional[Logger] = None, log_every: int = 100, ensemble_hparams=(),
                        buffer_hparams=("l1_alpha",), global_step: int = 0, progress: Optional[Callable] = None,
                        rank: int = 0, world: int = 1) -> int:
    """Train one ensemble for one pass over the ring (or ``n_batches``) with device-side sampling."""
    n = n_batches if n_batches is not None else ring.batches_per_epoch(batch_size * world)
    fused = trainer.kind.startswith("fused")
    xbuf = None
    if trainer.kind == "fused-sae" and getattr(trainer.impl, "use_graph", False) and trainer.es is None:
        xbuf = trainer.impl.x_static
    elif fused and ring.dtype == torch.bfloat16:
        xbuf = torch.empty(batch_size, ring.d, device=ring.device, dtype=ring.dtype)
    hp = trainer.hyperparams(ensemble_hparams, buffer_hparams, local=True)
    for i in range(n):
        with trace_range("sample"):
            x = ring.sample_shard(batch_size, rank, world, out=xbuf) if xbuf is not None else \
                ring.sample_shard(batch_size, rank, world)
        if fused and x.dtype != torch.bfloat16:
            x = x.to(torch.bfloat16)
        with trace_range("step"):
            trainer.step(x)
        global_step += 1
        if logger is not None and log_every and global_step % log_every == 0:
            logger.log(model_metric_names(trainer.name, hp, trainer.losses_host()), global_step)
        if progress is not None:
            progress(i + 1, n)
    return global_step


def unstacked_to_learned_dicts(trainer: EnsembleTrainer, args: dict, ensemble_hparams: Sequence[str],
                               buffer_hparams: Sequence[str]):
    """Reference big_sweep.py:245-268."""
    trainer.args.update(args or {})
    return trainer.to_learned_dicts(ensemble_hparams, buffer_hparams)


def filter_learned_dicts(learned_dicts, hyperparam_filters: dict):
    """Dicts whose hyper-parameters match (floats to rel 1e-3) -- reference big_sweep.py:61-74."""
    from math import isclose

    return [(ld, hp) for ld, hp in learned_dicts
            if all(isclose(hp[k], v, rel_tol=1e-3) if isinstance(v, float) else hp[k] == v
                   for k, v in hyperparam_filters.items())]


@torch.no_grad()
def log_standard_metrics(learned_dicts, sample: torch.Tensor, chunk_num: int, hyperparam_ranges: dict,
                         logger: Optional[Logger], image_dir: Optional[str] = None):
    """Per-dict ever-active counts on a sample (numbers to the logger) and, with
    ``image_dir``, MMCS-with-larger-dict grids and code-sparsity histograms as PNGs
    (reference big_sweep.py:87-158, wandb images there)."""
    from itertools import product

    from ..eval import metrics as M

    log = {}
    for ld, hp in learned_dicts:
        ld.to_device(sample.device)
        name = make_hyperparam_name(hp)
        n_act = int(M.batched_calc_feature_n_ever_active(ld, sample, threshold=1))
        log[name + "_n_active"] = n_act
        log[name + "_prop_active"] = n_act / ld.get_learned_dict().shape[0]
    if logger is not None:
        logger.log(log, chunk_num)
    if not image_dir:
        return log
    from ..eval import plotting as P

    os.makedirs(image_dir, exist_ok=True)
    l1_values = list(hyperparam_ranges.get("l1_alpha", []))
    sizes = list(hyperparam_ranges.get("dict_size", []))
    grid_hps = [k for k in hyperparam_ranges if k not in ("l1_alpha", "dict_size")]
    if len(sizes) > 1 and l1_values:
        for setting in product(*[hyperparam_ranges[h] for h in grid_hps]):
            base = dict(zip(grid_hps, setting))
            scores = np.zeros((len(l1_values), len(sizes) - 1))
            for i, l1 in enumerate(l1_values):
                small = filter_learned_dicts(learned_dicts, {**base, "l1_alpha": float(l1), "dict_size": sizes[0]})
                for j, size in enumerate(sizes[1:]):
                    large = filter_learned_dicts(learned_dicts, {**base, "l1_alpha": float(l1), "dict_size": size})
                    if small and large:
                        scores[i, j] = float(M.mcs_duplicates(small[0][0], large[0][0]).mean())
            img = P.plot_grid(scores, [f"{v:.1e}" for v in l1_values], sizes[1:], "l1_alpha", "dict_size",
                              cmap="viridis")
            img.save(os.path.join(image_dir, f"mmcs_grid_{chunk_num}_{make_hyperparam_name(base) or 'all'}.png"))
    for ld, hp in learned_dicts:
        img = P.plot_hist(M.mean_nonzero_activations(ld, sample).cpu(), "Mean nonzero activations", "Frequency",
                          bins=20)
        img.save(os.path.join(image_dir, f"sparsity_hist_{chunk_num}_{make_hyperparam_name(hp)}.png"))
    return log


def _load_chunk_into_ring(folder: ChunkFolder, handle, ring: DeviceRing, means: Optional[torch.Tensor]):
    host = folder.get(handle)
    ring.size = 0
    ring.head = 0
    dev = host.to(ring.device, non_blocking=True)
    if means is not None:
        dev = (dev.float() - means.to(ring.device)).to(ring.dtype)
    ring.push(dev)
    return dev.shape[0]


def sweep(ensemble_init_func, cfg, info: Optional[DistInfo] = None) -> List[Tuple[Any, dict]]:
    """Run a hyper-parameter sweep over the chunks in ``cfg.dataset_folder`` (reference big_sweep.py:341-429)."""
    info = info or init_distributed()
    device = info.device if info.device.type == "cuda" else torch.device(cfg.device if torch.cuda.is_available() else "cpu")
    torch.manual_seed(cfg.seed)
    np.random.seed(cfg.seed)
    os.makedirs(cfg.output_folder, exist_ok=True)
    os.makedirs(cfg.dataset_folder, exist_ok=True)

    # ---- data: existing chunks, synthetic generation, or harvest (reference init_*_dataset)
    if not [f for f in os.listdir(cfg.dataset_folder) if f.endswith(".pt")]:
        if info.is_main:
            _create_dataset(cfg, device)
        barrier(info)
    folder = ChunkFolder(cfg.dataset_folder)
    d = folder.meta(folder.indices[0])[0][1]
    cfg.activation_width = d

    ensembles, ensemble_hparams, buffer_hparams, hparam_ranges = ensemble_init_func(cfg)
    cfg.ensemble_hyperparams = list(ensemble_hparams)
    cfg.buffer_hyperparams = list(buffer_hparams)
    trainers: List[EnsembleTrainer] = []
    for gi, (models, sig, args, name) in enumerate(ensembles):
        if info.world_size > 1 and gi % info.world_size != info.rank:
            trainers.append(None)  # sweep sharding: this ensemble lives on another rank
            continue
        trainers.append(EnsembleTrainer(models, sig, lr=cfg.lr, batch_size=args.get("batch_size", cfg.batch_size),
                                        device=device, engine=cfg.engine, name=name, args=args,
                                        fista_iters=getattr(cfg, "fista_iters", 500),
                                        fista_backend=getattr(cfg, "fista_backend", "auto"),
                                        persist_hessian=getattr(cfg, "persist_hessian", False),
                                        basis_normalize=getattr(cfg, "basis_normalize", "column"),
                                        fista_eta=getattr(cfg, "fista_eta", "tracked"),
                                        use_graph=cfg.use_graph,
                                        objective=args.get("objective", "loss"),
                                        fista_loss_iters=int(args.get("fista_loss_iters", 50))))

    n_chunks = len(folder)
    chunk_order = np.random.permutation(folder.indices)
    chunk_order = np.tile(chunk_order, max(1, cfg.n_repetitions or 1))
    logger = Logger.from_config(cfg.log_dir or cfg.output_folder, cfg.use_wandb, 0, cfg.to_dict(), info.rank)

    # ---- resume
    state_path = os.path.join(cfg.output_folder, f"train_state_rank{info.rank}.pt")
    start, global_step, means = 0, 0, None
    if cfg.resume and os.path.exists(state_path):
        st = ckpt.load_training_state(state_path)
        start = st["extra"]["next_chunk"]
        global_step = st["extra"]["global_step"]
        chunk_order = np.array(st["extra"]["chunk_order"])
        means = st["extra"].get("means")
        for t, ts in zip(trainers, st["trainer"]["ensembles"]):
            if t is not None and ts is not None:
                t.load_state_dict(ts)
        ckpt.set_rng_state(st["rng"])

    rows_max = max(folder.meta(i)[0][0] for i in folder.indices)
    # fused kernels consume bf16 rows; the eager engine trains in fp32 on the fp16 chunk values
    any_fused = any(t is not None and t.kind.startswith("fused") for t in trainers)
    ring = DeviceRing(rows_max, d, device=device, dtype=torch.bfloat16 if any_fused else torch.float32,
                      seed=cfg.seed + info.rank)
    handle = folder.prefetch(int(chunk_order[start])) if start < len(chunk_order) else None
    learned_dicts: List[Tuple[Any, dict]] = []
    for i in range(start, len(chunk_order)):
        chunk_idx = int(chunk_order[i])
        t0 = time.time()
        with trace_range("load_chunk"):
            if cfg.center_activations and means is None:
                host = folder.load(chunk_idx).float()
                means = host.mean(0)
                torch.save(means, os.path.join(cfg.output_folder, "means.pt"))
            _load_chunk_into_ring(folder, handle, ring, means if cfg.center_activations else None)
        if i + 1 < len(chunk_order):  # stream the next chunk from disk while this one trains
            handle = folder.prefetch(int(chunk_order[i + 1]))
        for t in trainers:
            if t is None:
                continue
            global_step = ensemble_train_loop(t, ring, t.batch_size, None, logger, cfg.log_every,
                                              cfg.ensemble_hyperparams, cfg.buffer_hyperparams, global_step)
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        learned_dicts = []
        for t in trainers:
            if t is not None:
                learned_dicts.extend(t.to_learned_dicts(cfg.ensemble_hyperparams, cfg.buffer_hyperparams))
        logger.log({"chunk": i, "chunk_idx": chunk_idx, "chunk_seconds": time.time() - t0}, global_step)
        if learned_dicts and i % 10 == 0:  # reference cadence (big_sweep.py:416)
            sample = ring.view()[torch.randperm(ring.size, device=ring.device)[:2000]].float()
            log_standard_metrics(learned_dicts, sample, i, hparam_ranges, logger,
                                 os.path.join(cfg.output_folder, "images") if cfg.wandb_images else None)
        suffix = "" if info.world_size == 1 else f"_rank{info.rank}"
        if i == len(chunk_order) - 1 or (i + 1) in CHECKPOINT_COUNTS:
            it_folder = os.path.join(cfg.output_folder, f"_{i}")
            os.makedirs(it_folder, exist_ok=True)
            ckpt.save_learned_dicts(learned_dicts, os.path.join(it_folder, f"learned_dicts{suffix}.pt"))
            if info.is_main:
                cfg.to_yaml(os.path.join(it_folder, "config.yaml"))
        ckpt.save_training_state(state_path, {"ensembles": [t.state_dict() if t is not None else None
                                                            for t in trainers]},
                                 {"next_chunk": i + 1, "global_step": global_step,
                                  "chunk_order": chunk_order.tolist(), "means": means})
    logger.close()
    return learned_dicts


SYNTHETIC_MARKER = ".sc_synthetic_dataset"


def remove_synthetic_dataset(folder: str) -> bool:
    """Delete ``folder`` only if this package generated it (marker file present); a folder of
    harvested or user activations is never touched.  Returns True when something was removed."""
    import shutil

    if not os.path.isdir(folder):
        return False
    if not os.path.exists(os.path.join(folder, SYNTHETIC_MARKER)):
        raise RuntimeError(f"refusing to delete {folder!r}: it was not written by the synthetic dataset "
                           f"generator (no {SYNTHETIC_MARKER} marker)")
    shutil.rmtree(folder)
    return True


def _create_dataset(cfg, device):
    """Reference init_synthetic_dataset / init_model_dataset (big_sweep.py:271-338)."""
    from ..data.chunks import save_chunk

    if getattr(cfg, "use_synthetic_dataset", False):
        from ..data.synthetic import SparseMixDataset

        n_gt = getattr(cfg, "n_ground_truth_components", 512)
        gen = SparseMixDataset(cfg.activation_width, n_gt, getattr(cfg, "gen_batch_size", 4096),
                               getattr(cfg, "feature_num_nonzero", 10), getattr(cfg, "feature_prob_decay", 0.99),
                               getattr(cfg, "noise_magnitude_scale", 0.0), device,
                               sparse_component_covariance=None if getattr(cfg, "correlated_components", False)
                               else torch.eye(n_gt, device=device), seed=cfg.seed)
        rows = int(cfg.chunk_size_gb * 1024 ** 3 // (cfg.activation_width * 2))  # fp16 chunks (fix B#27)
        for i in range(cfg.n_chunks):
            parts, have = [], 0
            while have < rows:
                parts.append(gen.send(None).half())
                have += parts[-1].shape[0]
            save_chunk(torch.cat(parts)[:rows], cfg.dataset_folder, i)
        # marker: this folder holds generated chunks only (runners may delete it to regenerate)
        with open(os.path.join(cfg.dataset_folder, SYNTHETIC_MARKER), "w") as f:
            f.write("synthetic chunks written by sparse_coding__amd.train.sweep\n")
        torch.save({"feats": gen.sparse_component_dict.cpu(), "probs": gen.sparse_component_probs.cpu()},
                   os.path.join(cfg.output_folder, "generator.pt"))
    else:
        from ..data.harvest import setup_data

        setup_data(cfg.model_name, cfg.dataset_folder, cfg.layer, cfg.layer_loc, n_chunks=cfg.n_chunks,
                   chunk_size_gb=cfg.chunk_size_gb, device=device, center_dataset=cfg.center_dataset,
                   seed=cfg.seed)
