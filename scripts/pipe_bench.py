"""Step-GEMM timings for every (block shape, K pipeline) configuration (config 2 shapes).

  python scripts/pipe_bench.py       -> one JSON line per (kernel, cfg)
  PB_CFGS=1,5 PB_KERNELS=dec python scripts/pipe_bench.py   -> a subset
cfg = shape | pipe << 2 (ops/gemm.py SHAPES / PIPES).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from scripts.kernel_bench import timeit  # noqa: E402


def main():
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.models.signatures import FunctionalSAE
    from sparse_coding__amd.ops import gemm

    B, d, n, G = [int(v) for v in (os.environ.get("PB_SHAPE") or "2048,512,2048,8").split(",")]
    dev = "cuda"
    models = [FunctionalSAE.init(d, n, 1e-3 * (i + 1), device=dev) for i in range(G)]
    e = FusedSAEEnsemble(models, FunctionalSAE, batch_size=B, device=dev)
    x = (torch.randn(B, d, device=dev) * 0.4).to(torch.bfloat16)
    e.step_batch(x)
    fl = 2.0 * B * n * d * G
    kernels = {
        "enc": (lambda: gemm.encode_relu(x, e.enc_shadow, e.params["encoder_bias"], e.c, e.enc_part, None, None), fl),
        "enc_cnt": (lambda: gemm.encode_relu(x, e.enc_shadow, e.params["encoder_bias"], e.c, e.enc_part, e.cnt_part,
                                             None), fl),
        "dec": (lambda: gemm.decode_residual(e.c, e.dec_shadow, x, e.r, e.dec_part), fl),
        "dc": (lambda: gemm.code_grad(e.r, e.dec_shadow, e.c, e.l1, e.dpre, e.colpart), fl),
        "wgrad2": (lambda: gemm.weight_grads([[(e.c, e.r)], [(e.dpre, x)]], [e.g_dec, e.g_enc], 1e-6), 2 * fl),
    }
    cfgs = [int(c) for c in (os.environ.get("PB_CFGS") or "1,5,9,13,2,3,7,11,15").split(",")]
    only = set(filter(None, (os.environ.get("PB_KERNELS") or "").split(",")))
    for cfg in cfgs:
        for name, (fn, f) in kernels.items():
            if only and name not in only:
                continue
            if not gemm.shape_fits(cfg, B if name != "wgrad2" else n, n if name in ("enc", "enc_cnt", "dc") else d):
                continue
            with gemm.force_shape(cfg):
                try:
                    t = timeit(fn, iters=100, warmup=10)
                except Exception as ex:  # configuration not instantiated
                    print(json.dumps({"kernel": name, "cfg": cfg, "error": str(ex)[:80]}))
                    continue
            print(json.dumps({"kernel": name, "cfg": cfg, "shape": gemm.SHAPES[cfg & 3],
                              "pipe": gemm.PIPES[(cfg >> 2) & 3], "p32": bool(cfg & 16), "us": round(t, 2), "tflops": round(f / t / 1e6, 1)}),
                  flush=True)


if __name__ == "__main__":
    main()
