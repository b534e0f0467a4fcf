"""Attribute the gap between short (driver: --steps 20 --warmup 5) and long bench runs.

One process, the bench's headline engine (8 untied SAEs, d=512, n=2048, B=2048), ring source.
Measures, each with synchronize on both sides:
  * first / second / third replay of a freshly captured 8-step graph, without and with
    hipGraphUpload right after capture;
  * an 8-step replay right after a 50 ms idle GPU vs back-to-back;
  * 8 single-step replays vs one 8-step replay (replay-boundary gaps).
Prints one JSON line per measurement.
"""

import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import bench  # noqa: E402
from sparse_coding__amd.engine import fused  # noqa: E402
from sparse_coding__amd.engine.fused import FusedSAEEnsemble  # noqa: E402
from sparse_coding__amd.models.signatures import FunctionalSAE  # noqa: E402


def timeit(fn):
    torch.cuda.synchronize()
    t = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t)


def main():
    import numpy as np

    args = bench.parse(["--ring-rows", str(1 << 20)])
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    models = [FunctionalSAE.init(512, 2048, float(l), device=dev) for l in np.logspace(-4, -2, 8)]
    ring, _ = bench.build_ring(args, dev)
    eng = FusedSAEEnsemble(models, FunctionalSAE, lr=1e-3, batch_size=2048, device=dev)
    eng.enable_graph().attach_source(ring.graph_source(2048))
    up = fused._upload
    out = []
    for label, upload in (("no_upload", False), ("upload", True)):
        fused._upload = up if upload else (lambda g, d: None)
        pat = tuple([upload] + [False] * 7)  # a fresh pattern -> fresh graph per variant
        t = timeit(lambda: eng.prime_source(patterns=[pat]))
        rec = {"probe": "first_replays", "variant": label, "capture_ms": round(t, 3)}
        rec["replay_ms"] = [round(timeit(lambda: eng.step_source(8, pat)), 4) for _ in range(4)]
        out.append(rec)
    fused._upload = up
    pat = (True,) + (False,) * 7
    for _ in range(20):
        eng.step_source(8, pat)
    back = [round(timeit(lambda: eng.step_source(8, pat)), 4) for _ in range(5)]
    idle = []
    for _ in range(5):
        time.sleep(0.05)
        idle.append(round(timeit(lambda: eng.step_source(8, pat)), 4))
    out.append({"probe": "idle_50ms", "back_to_back_ms": back, "after_idle_ms": idle})
    eng.prime_source(patterns=[(True,), (False,)])
    for _ in range(3):
        for c in (True,) + (False,) * 7:
            eng.step_source(1, (c,))

    def singles():
        for c in (True,) + (False,) * 7:
            eng.step_source(1, (c,))

    s1 = [round(timeit(singles), 4) for _ in range(5)]
    s8 = [round(timeit(lambda: eng.step_source(8, pat)), 4) for _ in range(5)]
    # many groups back to back: steady-state per-step time
    t = timeit(lambda: [eng.step_source(8, pat) for _ in range(25)])
    out.append({"probe": "replay_gaps", "eight_single_ms": s1, "one_eight_ms": s8,
                "steady_ms_per_step_200": round(t / 200, 4)})
    for r in out:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
