"""FVU-vs-L0 curves of the L1 sweep on MI355X (the quality half of the headline metric).

Trains the reference's sweep -- 8 SAEs, l1 = logspace(-4, -2, 8) -- with the fused engine
on calibrated synthetic Pythia-70m-shaped activations (bench.py --act-norm), then scores
FVU and L0 on held-out rows exactly like ``plotting/fvu_sparsity_plot.py:104-185``
(``eval/metrics.py``).  Three sweeps: untied ratio 1 (the dictionary size of the
reference's plotted runs, dict 512), tied ratio 1 (the class of the shipped ``normal``
checkpoint) and untied ratio 4 (BASELINE config 2).  Writes one JSON line per model and a
PNG with the reference's SAE points read off ``output_basic_test/graphs/fistavnormal.png``
 for orientation -- those come from real Pythia-70m activations, so
the curves are comparable in shape, not point for point.

  python scripts/fvu_curve.py --steps 20000 --out gpurun_out/fvu_curve
"""

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

# Adam SAE ensemble, dict 512, Pythia-70m layer-2 residual
REF_SAE = [(2, 0.38), (9, 0.24), (24, 0.15), (50, 0.105), (118, 0.065), (232, 0.040), (337, 0.022), (406, 0.011)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20000)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--act-norm", type=float, default=9.0)
    ap.add_argument("--eval-rows", type=int, default=16384)
    ap.add_argument("--out", default="gpurun_out/fvu_curve")
    a = ap.parse_args()
    import bench
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.models.signatures import FunctionalSAE, FunctionalTiedSAE

    dev = "cuda:0"
    args = bench.parse(["--act-norm", str(a.act_norm), "--eval-rows", str(a.eval_rows)])
    ring, held = bench.build_ring(args, dev)
    held = held.float()
    l1s = np.logspace(-4, -2, 8)
    results = []
    for name, sig, ratio in (("untied_r1", FunctionalSAE, 1), ("tied_r1", FunctionalTiedSAE, 1),
                             ("untied_r4", FunctionalSAE, 4)):
        torch.manual_seed(0)
        models = [sig.init(512, 512 * ratio, float(l), device=dev) for l in l1s]
        eng = FusedSAEEnsemble(models, sig, lr=1e-3, batch_size=a.batch, device=dev).enable_graph()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            ring.sample(a.batch, out=eng.x_static)
            eng.step_static()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        q = bench.fvu_l0(eng.to_learned_dicts(dev), held)
        for l1, (l0, fvu) in zip(l1s, q):
            rec = {"sweep": name, "ratio": ratio, "l1": float(l1), "l0": round(l0, 2), "fvu": round(fvu, 4),
                   "steps": a.steps, "batch": a.batch, "train_s": round(el, 2)}
            results.append(rec)
            print(json.dumps(rec), flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out + ".json", "w") as f:
        json.dump({"act_norm": a.act_norm, "steps": a.steps, "batch": a.batch, "results": results,
                   "reference_plot_points": REF_SAE}, f, indent=1)
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt

        fig, ax = plt.subplots(figsize=(6, 4.5))
        for name in ("untied_r1", "tied_r1", "untied_r4"):
            pts = [(r["l0"], r["fvu"]) for r in results if r["sweep"] == name]
            ax.plot(*zip(*pts), "o-", label=f"MI355X {name}")
        ax.plot(*zip(*REF_SAE), "k^--", label="reference SAE (Pythia-70m, PLOT)")
        ax.set_xlabel("L0 (mean active features)")
        ax.set_ylabel("FVU")
        ax.set_xscale("log")
        ax.legend()
        fig.tight_layout()
        fig.savefig(a.out + ".png", dpi=110)
    except Exception as e:  # plotting is optional
        print(f"plot skipped: {e}", file=sys.stderr)


if __name__ == "__main__":
    main()
