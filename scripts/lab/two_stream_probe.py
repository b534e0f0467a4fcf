"""Probe: the headline step as TWO independent 4-model pipelines on two streams of one HIP graph.

The eight SAEs of the headline ensemble share only the input batch, so the step can run as two
4-model engines whose kernels interleave on the GPU: one half's HBM-bound step tail (Adam) can
overlap the other half's MFMA GEMMs, and each kernel's last-round tail is filled by the other
stream.  Compared here against the shipped single 8-model engine, both replaying 8-step graphs on a
static batch (no gather, no feature counting), same models and shapes.  Prints JSON lines.
"""

import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

from sparse_coding__amd.engine.fused import FusedSAEEnsemble  # noqa: E402
from sparse_coding__amd.models.signatures import FunctionalSAE  # noqa: E402

STEPS = 8


def timed(g, reps):
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t) / (reps * STEPS)


def main():
    import numpy as np

    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    l1s = np.logspace(-4, -2, 8)
    models = [FunctionalSAE.init(512, 2048, float(l), device=dev) for l in l1s]
    x = torch.randn(2048, 512, device=dev).to(torch.bfloat16)
    one = FusedSAEEnsemble(models, FunctionalSAE, lr=1e-3, batch_size=2048, device=dev, track_feature_counts=False)
    halves = [FusedSAEEnsemble(models[:4], FunctionalSAE, lr=1e-3, batch_size=2048, device=dev,
                               track_feature_counts=False),
              FusedSAEEnsemble(models[4:], FunctionalSAE, lr=1e-3, batch_size=2048, device=dev,
                               track_feature_counts=False)]
    for e in [one] + halves:  # eager warmup (kernel loads, tail partials)
        e._tail_ready()
        e._step_kernels(x, False)
    torch.cuda.synchronize()

    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1):
        for _ in range(STEPS):
            one._step_kernels(x, False)

    side = [torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)]
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2):
        main_s = torch.cuda.current_stream()
        for _ in range(STEPS):
            for s in side:
                s.wait_stream(main_s)
            for s, e in zip(side, halves):
                with torch.cuda.stream(s):
                    e._step_kernels(x, False)
            for s in side:
                main_s.wait_stream(s)

    # the same two halves serialised on one stream (the split's own cost, no overlap)
    g3 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g3):
        for _ in range(STEPS):
            for e in halves:
                e._step_kernels(x, False)

    res = {}
    for name, g in (("one_8model", g1), ("two_streams", g2), ("two_serial", g3)):
        res[name] = [round(timed(g, 25), 4) for _ in range(3)]
    for name in list(res):
        print(json.dumps({"variant": name, "ms_per_step": res[name]}), flush=True)


if __name__ == "__main__":
    main()
