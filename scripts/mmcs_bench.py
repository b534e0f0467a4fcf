"""Max-cosine-similarity (MMCS) timing: the EPI_ROWMAX kernel vs torch.

For two unit-norm dictionaries [n, d] the reference computes ``(A @ B.T).max(-1)``
(standard_metrics.py:268-301), materialising the [n, n] similarity matrix.  The fused
kernel keeps each 128x128 tile in registers and writes one partial max per row and
64-column wave tile.  Prints one JSON line per shape.
"""

from __future__ import annotations

import json
import time

import torch

from sparse_coding__amd.ops import gemm


def _time(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    torch.manual_seed(0)
    for n, d in ((4096, 512), (16384, 512), (32768, 2048)):
        a = torch.nn.functional.normalize(torch.randn(n, d, device="cuda"), dim=-1)
        b = torch.nn.functional.normalize(torch.randn(n, d, device="cuda"), dim=-1)
        ab, bb = a.to(torch.bfloat16), b.to(torch.bfloat16)
        exact = (a @ b.T).max(-1).values
        fused = gemm.rowmax_nt(ab, bb)
        err = float((fused - exact).abs().max())
        t_fused = _time(lambda: gemm.rowmax_nt(ab, bb))
        t_f32 = _time(lambda: (a @ b.T).max(-1).values)
        t_bf16 = _time(lambda: (ab @ bb.T).max(-1).values)
        flop = 2.0 * n * n * d
        extra = {}
        try:  # 256x256 blocks (128x64 per wave)
            extra["fused_256_err"] = round(float((gemm.rowmax_nt(ab, bb, cfg=3) - exact).abs().max()), 5)
            extra["fused_256_ms"] = round(_time(lambda: gemm.rowmax_nt(ab, bb, cfg=3)), 3)
        except RuntimeError as e:
            extra["fused_256"] = str(e)[:120]
        print(json.dumps({"n1": n, "n2": n, "d": d, "fused_ms": round(t_fused, 3), "torch_fp32_ms": round(t_f32, 3),
                          "torch_bf16_ms": round(t_bf16, 3), "fused_tflops": round(flop / t_fused / 1e9, 1),
                          "max_abs_err_vs_fp32": round(err, 5), **extra}), flush=True)


if __name__ == "__main__":
    main()
