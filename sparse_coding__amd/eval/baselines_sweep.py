"""Baseline dictionaries per layer, matched in sparsity to a trained SAE.

Reference: ``sweep_baselines.py:17-160`` -- for every (layer, location): streaming
PCA (full and top-k at the SAE's L0), ICA (+ top-k), a random dictionary and
identity-ReLU, one process per GPU over layers.  Here:

* PCA covariance accumulates with GEMMs on the device (``BatchedPCA``), ICA fits on
  the CPU (sklearn, float64) and is then a pure tensor encoder;
* every baseline is written with the safe, reference-layout checkpoint writer
  (``[(dict, {"kind": ..., "sparsity": k})]``) so it loads with
  ``load_learned_dicts`` (``weights_only=True``);
* the target sparsity comes from a reference SAE checkpoint (``match_dicts`` +
  ``match_index``, reference uses entry 7 of the tied r1 sweep) or a fixed number;
* ``run_all`` fans layers out over GPUs with one spawned process each.
"""

from __future__ import annotations

import os
from typing import List, Optional, Sequence

import torch

from ..baselines.ica import ICAEncoder, NMFEncoder
from ..baselines.pca import BatchedPCA
from ..models.learned_dict import IdentityReLU, RandomDict
from ..utils.checkpoint import load_learned_dicts, save_learned_dicts
from .metrics import mean_nonzero_activations


def matched_sparsity(match_dicts: str, index: int, activations: torch.Tensor) -> int:
    ld, hp = load_learned_dicts(match_dicts)[index]
    ld.to_device(activations.device)
    return int(round(float(mean_nonzero_activations(ld, activations.float()).sum())))


def run_layer_baselines(layer: int, layer_locs: Sequence[str], chunks_folder: str, output_folder: str,
                        sparsity: int = 50, device="cpu", remake: bool = False, match_dicts: Optional[str] = None,
                        match_index: int = 7, pca_batch_size: int = 8192, ica_rows: int = 0, with_nmf: bool = False,
                        seed: int = 0) -> List[str]:
    written = []
    for loc in layer_locs:
        name = f"l{layer}_{loc}"
        out = os.path.join(output_folder, name)
        os.makedirs(out, exist_ok=True)
        chunk = torch.load(os.path.join(chunks_folder, name, "0.pt"), weights_only=True, map_location="cpu")
        acts = chunk.to(device=device, dtype=torch.float32)
        d = acts.shape[1]
        k = matched_sparsity(match_dicts, match_index, acts) if match_dicts else int(sparsity)

        def save(fname, ld, kind):
            path = os.path.join(out, fname)
            save_learned_dicts([(ld, {"kind": kind, "sparsity": k, "layer": layer, "layer_loc": loc})], path)
            written.append(path)

        def todo(fname):
            return remake or not os.path.exists(os.path.join(out, fname))

        if todo("pca.pt"):
            pca = BatchedPCA(d, device)
            with torch.no_grad():
                for i in range(0, acts.shape[0], pca_batch_size):
                    pca.train_batch(acts[i:i + pca_batch_size])
            save("pca.pt", pca.to_learned_dict(d), "pca")
            save("pca_topk.pt", pca.to_topk_dict(k), "pca_topk")
        if todo("ica.pt"):
            ica = ICAEncoder(d, seed=seed)
            rows = acts[:ica_rows] if ica_rows else acts
            ica.train(rows)
            save("ica.pt", ica, "ica")
            save("ica_topk.pt", ica.to_topk_dict(k), "ica_topk")
        if with_nmf and todo("nmf_topk.pt"):
            nmf = NMFEncoder(d, seed=seed)
            nmf.train(acts[:ica_rows] if ica_rows else acts)
            save("nmf_topk.pt", nmf.to_topk_dict(k), "nmf_topk")
        if todo("random.pt"):
            save("random.pt", RandomDict(d, generator=torch.Generator().manual_seed(seed)), "random")
        if todo("identity_relu.pt"):
            save("identity_relu.pt", IdentityReLU(d), "identity_relu")
    return written


def _worker(args):
    layer, kw = args
    return run_layer_baselines(layer, **kw)


def run_all(layers: Sequence[int], layer_locs: Sequence[str], chunks_folder: str, output_folder: str,
            sparsity: int = 50, devices: Optional[Sequence[str]] = None, **kw) -> List[str]:
    """One spawned process per layer, round-robin over ``devices``."""
    import torch.multiprocessing as mp

    devices = list(devices or ([f"cuda:{i}" for i in range(torch.cuda.device_count())] or ["cpu"]))
    tasks = [(L, dict(layer_locs=list(layer_locs), chunks_folder=chunks_folder, output_folder=output_folder,
                      sparsity=sparsity, device=devices[i % len(devices)], **kw)) for i, L in enumerate(layers)]
    if len(tasks) == 1:
        return _worker(tasks[0])
    with mp.get_context("spawn").Pool(min(len(tasks), len(devices))) as pool:
        return [p for r in pool.map(_worker, tasks) for p in r]
