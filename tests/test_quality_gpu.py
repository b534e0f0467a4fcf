"""Training quality of the bf16 fused engine against the reference's fp32 math over a training horizon.

The fused engine computes in bf16 MFMA (fp32 masters, fp32 Adam); the reference trains in fp32
(``autoencoders/sae_ensemble.py:53-77`` under ``vmap(grad)`` + Adam, reproduced by
``engine/ensemble.py``'s FunctionalEnsemble).  Both train the same models on the same batches for
500 steps; per model the held-out FVU and mean L0 (``standard_metrics.py:303-312``) must agree
within 5 % relative.  The full-size comparison (headline config, 3000 steps) is
``scripts/quality_pin.py`` -> ``profiles/r5/quality/``.
"""

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def test_bf16_fused_matches_fp32_reference_training_quality():
    from sparse_coding__amd.data.synthetic import RandomDatasetGenerator
    from sparse_coding__amd.engine.ensemble import FunctionalEnsemble
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.engine.optim import adam
    from sparse_coding__amd.eval.metrics import fraction_variance_unexplained, mean_l0
    from sparse_coding__amd.models.signatures import FunctionalSAE

    torch.manual_seed(0)
    d, n, B, steps = 512, 1024, 512, 500
    l1s = [1e-4, 3e-4, 1e-3, 3e-3]
    gen = RandomDatasetGenerator(activation_dim=d, n_ground_truth_components=4 * d, batch_size=B,
                                 feature_num_nonzero=32, feature_prob_decay=0.999, correlated=False,
                                 device=DEV, seed=11)
    probe = gen.send(None)
    scale = 9.0 / float(probe.norm(dim=-1).mean())  # the bench's row scale
    models = [FunctionalSAE.init(d, n, l1, device=DEV) for l1 in l1s]
    ref = FunctionalEnsemble([({k: v.clone() for k, v in p.items()}, b) for p, b in models], FunctionalSAE, adam,
                             {"lr": 1e-3}, device=DEV)
    fused = FusedSAEEnsemble(models, FunctionalSAE, lr=1e-3, batch_size=B, device=DEV)
    for _ in range(steps):
        x = (gen.send(None) * scale).to(torch.bfloat16)  # both engines see the same bf16 rows
        ref.step_batch(x.float())
        fused.step_batch(x)
    held = torch.cat([gen.send(None) for _ in range(8)]) * scale
    held = held.to(torch.bfloat16).float()
    torch.cuda.synchronize()
    got = fused.to_learned_dicts(DEV)
    want = ref.to_learned_dicts(DEV)
    rows = []
    for g, (a, b) in enumerate(zip(got, want)):
        fa, fb = float(fraction_variance_unexplained(a, held)), float(fraction_variance_unexplained(b, held))
        la, lb = float(mean_l0(a, held)), float(mean_l0(b, held))
        rows.append((l1s[g], fa, fb, la, lb))
    msg = "\n".join(f"l1={l:.0e}: fvu bf16 {fa:.4f} fp32 {fb:.4f} | L0 bf16 {la:.2f} fp32 {lb:.2f}"
                    for l, fa, fb, la, lb in rows)
    for l, fa, fb, la, lb in rows:
        assert abs(fa - fb) <= 0.05 * fb, msg
        assert abs(la - lb) <= 0.05 * lb, msg
    # and the sweep actually spans sparsity (the comparison is not between dead models)
    assert rows[0][3] > 2 * rows[-1][3] > 0, msg
