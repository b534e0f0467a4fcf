"""End to end on one MI355X: harvest -> HBM ring -> fused 8-model sweep -> FVU/L0 -> checkpoint.

The reference's pipeline (activation_dataset.setup_data -> big_sweep.sweep ->
plotting/fvu_sparsity_plot.generate_scores) with every stage on the device:

1. random-init Pythia-70m (GPT-NeoX, bf16; no network for weights) runs synthetic
   Zipf-distributed 256-token sequences; the layer-2 residual stream goes straight into a
   DeviceRing (no host round trip);
2. an 8-way L1 sweep (logspace(-4, -2, 8)) of untied SAEs, ratio 4, trains with the fused
   gfx950 engine (one HIP graph per step) on batches gathered from the ring;
3. FVU and L0 per model on held-out harvested rows (eval/metrics, the reference formulas);
4. the dictionaries are written as a reference-layout learned_dicts.pt and read back with
   the safe loader, and predict() of the reloaded dicts reproduces the in-memory FVU.

  python scripts/e2e_pythia70m.py --rows 2000000 --steps 5000 --out gpurun_out/e2e
"""

import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_000_000)
    ap.add_argument("--steps", type=int, default=5000)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--act-norm", type=float, default=9.0,
                    help="rescale rows to this mean norm (a trained Pythia-70m layer-2 residual's); 0 = keep")
    ap.add_argument("--out", default="gpurun_out/e2e")
    ap.add_argument("--keep-ckpt", action="store_true", help="write learned_dicts.pt into --out (64 MB)")
    a = ap.parse_args()
    from sparse_coding__amd.data.harvest import ActivationHarvester, build_model, harvest_to_ring, synthetic_token_batches
    from sparse_coding__amd.data.ring import DeviceRing
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.eval.metrics import fraction_variance_unexplained, mean_l0
    from sparse_coding__amd.models.signatures import FunctionalSAE
    from sparse_coding__amd.utils import checkpoint as ckpt

    dev = "cuda:0"
    os.makedirs(a.out, exist_ok=True)
    rec = {"model": "pythia-70m (random init, bf16)", "layer": 2, "layer_loc": "residual"}
    # 1. harvest
    lm = build_model("pythia-70m", device=dev, dtype=torch.bfloat16, seed=0)
    h = ActivationHarvester(lm, [2], "residual")
    ring = DeviceRing(a.rows, 512, device=dev, seed=1)
    toks = synthetic_token_batches(50304, batch=64, seq_len=256, seed=0, device=dev)
    t0 = time.perf_counter()
    harvest_to_ring(h, toks, {2: ring}, a.rows, device=dev)
    torch.cuda.synchronize()
    rec["harvest_rows"] = ring.size
    rec["harvest_s"] = round(time.perf_counter() - t0, 2)
    held = h.run(next(toks).to(dev))[2][:16384].float()
    h.close()
    del lm
    # a random-init residual stream's scale differs from a trained model's: report it and
    # rescale (in place, in the ring) so the l1 range lands on the same part of the curve
    norm = float(held.norm(dim=-1).mean())
    rec["raw_mean_row_norm"] = round(norm, 3)
    if a.act_norm > 0:
        s = a.act_norm / norm
        ring.view().mul_(s)
        held *= s
        rec["rescaled_to"] = a.act_norm
    # 2. train
    torch.manual_seed(0)
    l1s = np.logspace(-4, -2, 8)
    models = [FunctionalSAE.init(512, 2048, float(l), device=dev) for l in l1s]
    from sparse_coding__amd.engine.graph_plan import chunks, count_pattern

    # the bench's step: multi-step HIP graphs with the ring gather inside (the fused tail fetches
    # each next batch)
    eng = FusedSAEEnsemble(models, FunctionalSAE, lr=1e-3, batch_size=a.batch, device=dev).enable_graph()
    eng.attach_source(ring.graph_source(a.batch))
    groups = list(chunks(a.steps, 8))
    eng.prime_source(patterns=[count_pattern(s, 8) for s in sorted(set(groups))])
    t0 = time.perf_counter()
    for s in groups:
        eng.step_source(s, count_pattern(s, 8))
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    rec.update(train_steps=a.steps, train_s=round(el, 2), train_act_per_s=round(a.steps * a.batch / el, 1))
    # 3. evaluate
    lds = eng.to_learned_dicts(dev)
    scores = [(float(mean_l0(ld, held)), float(fraction_variance_unexplained(ld, held))) for ld in lds]
    fvu_k, l0_k = eng.evaluate(held)  # the kernels' own epilogue partials
    rec["fvu_at_l0"] = [{"l1": float(l), "l0": round(s[0], 2), "fvu": round(s[1], 4),
                         "fvu_kernel": round(float(f), 4), "l0_kernel": round(float(z), 2)}
                        for l, s, f, z in zip(l1s, scores, fvu_k.cpu(), l0_k.cpu())]
    # 4. checkpoint round trip (reference layout, safe loader)
    # (64 MB of fp32 dictionaries: kept out of --out unless --keep-ckpt, so a results directory
    # stays small enough to copy back)
    path = os.path.join(a.out if a.keep_ckpt else tempfile.mkdtemp(), "learned_dicts.pt")
    ckpt.save_learned_dicts([(ld, {"dict_size": 2048, "l1_alpha": float(l)})
                             for ld, l in zip(eng.to_learned_dicts("cpu"), l1s)], path)
    back = ckpt.load_learned_dicts(path)
    re = []
    for (ld, hp), s in zip(back, scores):
        ld.to_device(dev)
        re.append(abs(float(fraction_variance_unexplained(ld, held)) - s[1]))
    rec["checkpoint"] = {"path": path, "classes": sorted({type(ld).__name__ for ld, _ in back}),
                         "max_fvu_diff_after_reload": float(max(re))}
    print(json.dumps(rec), flush=True)
    with open(os.path.join(a.out, "e2e.json"), "w") as f:
        json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
