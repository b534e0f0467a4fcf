"""Minimal ensemble example (reference ``ensemble_training_example.py``): five SAEs with
log-spaced L1 train together on a correlated synthetic generator; MMCS with the
ground-truth features is printed every 100 steps.

On a GPU the ensemble runs on the fused gfx950 step (``EnsembleTrainer`` picks it);
on CPU it falls back to the eager ``FunctionalEnsemble``.

    python examples/ensemble_training_example.py [--steps 1000]
"""

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

from sparse_coding__amd.data.synthetic import RandomDatasetGenerator  # noqa: E402
from sparse_coding__amd.engine.trainer import EnsembleTrainer  # noqa: E402
from sparse_coding__amd.models.signatures import FunctionalSAE  # noqa: E402


def mmcs(truth, dictionary):
    """Mean over learned atoms of the best cosine match to a true feature."""
    return (truth @ dictionary.T).max(dim=0).values.mean()


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=1000)
    p.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    p.add_argument("--d", type=int, default=512)
    p.add_argument("--n", type=int, default=2048)
    p.add_argument("--batch", type=int, default=256)
    a = p.parse_args(argv)
    torch.manual_seed(0)
    gen = RandomDatasetGenerator(a.d, 1024, a.batch, 5, 0.99, True, a.device)
    base = 10 ** (1 / 4)
    l1 = [base ** i for i in range(-16, -11)]
    models = [FunctionalSAE.init(a.d, a.n, x) for x in l1]
    tr = EnsembleTrainer(models, FunctionalSAE, lr=1e-3, batch_size=a.batch, device=a.device)
    print(f"engine: {tr.kind} ({tr.engine_reason})")
    for i in range(a.steps):
        x = next(gen)
        tr.step(x.to(torch.bfloat16) if tr.kind.startswith("fused") else x)
        if i % 100 == 0 or i == a.steps - 1:
            dicts = [ld.get_learned_dict().to(gen.feats.device) for ld, _ in tr.to_learned_dicts([], [])]
            print(f"Step {i}\n    Losses: {tr.last_losses['loss'].tolist()}\n"
                  f"    MMCS: {[round(float(mmcs(gen.feats, D)), 4) for D in dicts]}")
    return tr


if __name__ == "__main__":
    main()
