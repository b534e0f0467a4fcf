"""What a 20-step timed region measures after different histories, in ONE process (bench engine,
8-step graph groups): right after a long run, after idle gaps of 1 / 10 / 100 ms, after a GEMM-loop
settle, after a settle of the training step's own graph replayed on a scratch engine.
Prints one JSON line per scenario (ms per step of the 20 timed steps, host clock, synchronize on
both sides)."""

import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import bench  # noqa: E402
from sparse_coding__amd.engine.fused import FusedSAEEnsemble  # noqa: E402
from sparse_coding__amd.engine.graph_plan import count_pattern  # noqa: E402
from sparse_coding__amd.models.signatures import FunctionalSAE  # noqa: E402


def main():
    args = bench.parse(["--ring-rows", str(1 << 20)])
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    mk = lambda: [FunctionalSAE.init(512, 2048, float(l), device=dev) for l in np.logspace(-4, -2, 8)]  # noqa: E731
    ring, _ = bench.build_ring(args, dev)
    eng = FusedSAEEnsemble(mk(), FunctionalSAE, lr=1e-3, batch_size=2048, device=dev)
    eng.enable_graph().attach_source(ring.graph_source(2048))
    scratch = FusedSAEEnsemble(mk(), FunctionalSAE, lr=1e-3, batch_size=2048, device=dev)
    scratch.enable_graph().attach_source(ring.graph_source(2048))
    pat4, pat8 = count_pattern(4), count_pattern(8)
    eng.prime_source(patterns=[pat4, pat8])
    scratch.prime_source(patterns=[pat8])

    def timed20():
        torch.cuda.synchronize()
        t = time.perf_counter()
        eng.step_source(8, pat8)
        eng.step_source(8, pat8)
        eng.step_source(4, pat4)
        torch.cuda.synchronize()
        return round(1e3 * (time.perf_counter() - t) / 20, 4)

    def steps(n):
        for _ in range(n // 8):
            eng.step_source(8, pat8)

    out = []
    eng.step_source(4, pat4)
    out.append(("cold_after_capture", timed20()))
    steps(400)
    out.append(("after_400_steps", timed20()))
    for idle in (1, 10, 100, 1000):
        steps(400)
        torch.cuda.synchronize()
        time.sleep(idle / 1e3)
        out.append((f"after_idle_{idle}ms", timed20()))
    time.sleep(0.5)
    r = bench.settle_clocks(dev, 150)
    out.append(("gemm_settle_150ms_synced", timed20()))
    time.sleep(0.5)
    from sparse_coding__amd.ops import gemm as gemm_ops
    a = torch.randn(2048, 512, device=dev).to(torch.bfloat16)
    b = torch.randn(8, 2048, 512, device=dev).to(torch.bfloat16)
    o = torch.empty(8, 2048, 2048, device=dev, dtype=torch.bfloat16)
    torch.cuda.synchronize()
    for _ in range(3500):
        gemm_ops.matmul_nt(a, b, o)
    out.append(("gemm_settle_3500_unsynced", timed20()))
    time.sleep(0.5)
    for _ in range(60):  # ~150 ms of the step itself on a scratch engine (its own parameters)
        scratch.step_source(8, pat8)
    out.append(("scratch_step_settle_480", timed20()))
    time.sleep(0.5)
    for _ in range(60):
        scratch.step_source(8, pat8)
    torch.cuda.synchronize()
    eng.step_source(4, pat4)  # + warmup 4 steps of the real engine
    out.append(("scratch_settle_then_warm4", timed20()))
    for k, v in out:
        print(json.dumps({"scenario": k, "ms_per_step": v}), flush=True)
    print(json.dumps({"gemm_settle": r}))


if __name__ == "__main__":
    main()
