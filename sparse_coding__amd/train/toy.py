"""Toy-model replication: recover known sparse features from synthetic data.

Reference: ``replicate_toy_models.py`` -- ``AutoEncoder`` (Linear+ReLU encoder,
bias-free decoder with columns re-normalised each forward, orthogonal init), loss
``MSE + l1 * mean_b |c|_1 / n``, trained one (l1, ratio) cell at a time, then MMCS
with the ground truth, dead neurons, running reconstruction loss, heat maps, and
MMCS of each dictionary with the next larger one.

MI355X design: the whole grid trains at once -- one ensemble per dictionary ratio,
all L1 values stacked -- on one shared generator stream, so every cell sees the
same batches (the reference shares the generator object across serial runs).
``engine="module"`` keeps the reference's exact per-cell ``nn.Module`` training
(weight projection instead of normalisation-in-the-loss) for parity studies.
Results are saved without pickle: ``results.npz`` + decoder tensors + config.yaml.
"""

from __future__ import annotations

import itertools
import os
from datetime import datetime
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.nn as nn

from ..data.synthetic import RandomDatasetGenerator
from ..engine.trainer import EnsembleTrainer
from ..models.signatures import FunctionalSAE
from ..utils.config import ToyArgs


class AutoEncoder(nn.Module):
    """Reference toy ``AutoEncoder`` (replicate_toy_models.py:208-229)."""

    def __init__(self, activation_size, n_dict_components):
        super().__init__()
        self.encoder = nn.Sequential(nn.Linear(activation_size, n_dict_components), nn.ReLU())
        self.decoder = nn.Linear(n_dict_components, activation_size, bias=False)
        nn.init.orthogonal_(self.decoder.weight)

    def forward(self, x):
        c = self.encoder(x)
        with torch.no_grad():
            self.decoder.weight.data = nn.functional.normalize(self.decoder.weight.data, dim=0)
        return self.decoder(c), c

    @property
    def device(self):
        return next(self.parameters()).device


def cosine_sim(a, b) -> np.ndarray:
    a = torch.as_tensor(np.asarray(a) if isinstance(a, np.ndarray) else a.detach()).float()
    b = torch.as_tensor(np.asarray(b) if isinstance(b, np.ndarray) else b.detach()).float().to(a.device)
    a = a / a.norm(dim=1, keepdim=True)
    b = b / b.norm(dim=1, keepdim=True)
    return (a @ b.T).cpu().numpy()


def mean_max_cosine_similarity(ground_truth_features, learned_dictionary) -> float:
    """For each ground-truth feature, the best-matching learned atom; averaged."""
    return float(cosine_sim(ground_truth_features, learned_dictionary).max(axis=1).mean())


@torch.no_grad()
def get_n_dead_neurons(encode, data_generator, n_batches: int = 10) -> int:
    acts = torch.cat([encode(next(data_generator)) for _ in range(n_batches)])
    return int((acts.mean(0) == 0).sum())


def compare_mmcs_with_larger_dicts(small: torch.Tensor, larger: List[torch.Tensor]) -> float:
    """Mean over atoms of ``small`` and over ``larger`` dicts of the best cosine match."""
    return float(np.mean([cosine_sim(small, big).max(axis=1) for big in larger]))


def run_single_go(cfg: ToyArgs, data_generator: Optional[RandomDatasetGenerator] = None):
    """One (l1, ratio) cell with the reference module and loss."""
    device = torch.device(cfg.device)
    gen = data_generator or RandomDatasetGenerator(cfg.activation_dim, cfg.n_ground_truth_components, cfg.batch_size,
                                                   cfg.feature_num_nonzero, cfg.feature_prob_decay,
                                                   cfg.correlated_components, device, seed=cfg.seed)
    ae = AutoEncoder(cfg.activation_dim, cfg.n_components_dictionary).to(device)
    opt = torch.optim.Adam(ae.parameters(), lr=cfg.lr)
    running, horizon = 0.0, 1000
    for _ in range(cfg.epochs):
        batch = next(gen)
        batch = batch + cfg.noise_level * torch.randn_like(batch)
        opt.zero_grad()
        x_hat, c = ae(batch)
        l_rec = torch.nn.functional.mse_loss(x_hat, batch)
        loss = l_rec + cfg.l1_alpha * c.abs().sum(1).mean() / c.size(1)
        loss.backward()
        opt.step()
        running = running * (horizon - 1) / horizon + float(l_rec.detach()) / horizon
    d = ae.decoder.weight.data.t()
    mmcs = mean_max_cosine_similarity(gen.feats, d)
    dead = get_n_dead_neurons(lambda x: ae.encoder(x), gen)
    return mmcs, ae, dead, running


def run_toy_grid(cfg: ToyArgs, l1_range: List[float], ratios: List[float], engine: str = "ensemble",
                 data_generator: Optional[RandomDatasetGenerator] = None):
    """Returns (mmcs [L, R], dead [L, R], recon [L, R], dicts[L][R])."""
    device = torch.device(cfg.device)
    gen = data_generator or RandomDatasetGenerator(cfg.activation_dim, cfg.n_ground_truth_components, cfg.batch_size,
                                                   cfg.feature_num_nonzero, cfg.feature_prob_decay,
                                                   cfg.correlated_components, device, seed=cfg.seed)
    L, R = len(l1_range), len(ratios)
    mmcs, dead, recon = np.zeros((L, R)), np.zeros((L, R)), np.zeros((L, R))
    dicts: List[List[Optional[torch.Tensor]]] = [[None] * R for _ in range(L)]
    if engine == "module":
        for (i, l1), (j, r) in itertools.product(enumerate(l1_range), enumerate(ratios)):
            cfg.l1_alpha, cfg.learned_dict_ratio = l1, r
            cfg.n_components_dictionary = int(cfg.n_ground_truth_components * r)
            m, ae, dn, rl = run_single_go(cfg, gen)
            mmcs[i, j], dead[i, j], recon[i, j] = m, dn, rl
            dicts[i][j] = ae.decoder.weight.detach().t().cpu()
        return mmcs, dead, recon, dicts
    # ensemble engine: all L1 values of one ratio in one ensemble; the reference's l1/n
    # scaling is folded into each model's l1_alpha
    trainers = []
    for r in ratios:
        n = int(cfg.n_ground_truth_components * r)
        models = [FunctionalSAE.init(cfg.activation_dim, n, l1 / n) for l1 in l1_range]
        trainers.append(EnsembleTrainer(models, FunctionalSAE, lr=cfg.lr, batch_size=cfg.batch_size, device=device,
                                        use_graph=device.type == "cuda"))
    run_rec = [torch.zeros(L, device=device) for _ in ratios]
    horizon = 1000
    for _ in range(cfg.epochs):
        batch = next(gen)
        if cfg.noise_level:
            batch = batch + cfg.noise_level * torch.randn_like(batch)
        xb = batch.to(torch.bfloat16) if any(t.kind.startswith("fused") for t in trainers) else None
        for j, t in enumerate(trainers):
            t.step(xb if t.kind.startswith("fused") else batch)
            rec = t.last_losses.get("l_reconstruction", t.last_losses["loss"])
            run_rec[j].mul_((horizon - 1) / horizon).add_(rec.float() / horizon)
    for j, t in enumerate(trainers):
        for i, (ld, _) in enumerate(t.to_learned_dicts([], [])):
            D = ld.get_learned_dict()
            dicts[i][j] = D
            mmcs[i, j] = mean_max_cosine_similarity(gen.feats.cpu(), D)
            ld.to_device(device)
            dead[i, j] = get_n_dead_neurons(lambda x: ld.encode(x.float()), gen)
            recon[i, j] = float(run_rec[j][i])
    return mmcs, dead, recon, dicts


def main(argv=None, engine: str = "ensemble"):
    from ..eval.plotting import plot_mat

    cfg = ToyArgs.from_cli(argv)
    torch.manual_seed(cfg.seed)
    np.random.seed(cfg.seed)
    l1_range = [cfg.l1_exp_base ** e for e in range(cfg.l1_exp_low, cfg.l1_exp_high)]
    ratios = [cfg.dict_ratio_exp_base ** e for e in range(cfg.dict_ratio_exp_low, cfg.dict_ratio_exp_high)]
    print("l1 values:", l1_range)
    print("dict ratios:", ratios)
    mmcs, dead, recon, dicts = run_toy_grid(cfg, l1_range, ratios, engine)
    out = os.path.join(cfg.output_folder, datetime.now().strftime("%Y%m%d-%H%M%S"))
    os.makedirs(out, exist_ok=True)
    plot_mat(mmcs, l1_range, ratios, save_folder=out, title="Mean Max Cosine Similarity w/ True",
             save_name="mmcs_matrix.png")
    plot_mat(np.clip(dead, 0, 100), l1_range, ratios, save_folder=out, title="Dead Neurons",
             save_name="dead_neurons_matrix.png")
    plot_mat(recon, l1_range, ratios, save_folder=out, title="Reconstruction Loss", save_name="recon_loss_matrix.png")
    larger = np.zeros_like(mmcs)
    for i, j in itertools.product(range(len(l1_range)), range(len(ratios) - 1)):
        larger[i, j] = compare_mmcs_with_larger_dicts(dicts[i][j], [dicts[i][j + 1]])
    plot_mat(larger, l1_range, ratios, save_folder=out, title="Average mmcs with larger dicts",
             save_name="av_mmcs_with_larger_dicts.png")
    np.savez(os.path.join(out, "results.npz"), mmcs=mmcs, dead=dead, recon=recon, mmcs_larger=larger,
             l1=np.array(l1_range), ratios=np.array(ratios))
    torch.save({"dicts": dicts}, os.path.join(out, "dicts.pt"))
    cfg.to_yaml(os.path.join(out, "config.yaml"))
    return out


if __name__ == "__main__":
    main()
