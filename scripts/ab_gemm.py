"""Interleaved A/B timing of the step GEMMs over (block shape, K pipeline) configs:
R rounds x every config, median per config (one process, so clock/DVFS drift hits every
config alike -- cdna_hip_programming.md rule 24)."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def t_once(fn, iters=30):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.models.signatures import FunctionalSAE
    from sparse_coding__amd.ops import gemm

    B, d, n, G = [int(v) for v in (os.environ.get("PB_SHAPE") or "2048,512,2048,8").split(",")]
    dev = "cuda"
    torch.manual_seed(0)
    models = [FunctionalSAE.init(d, n, 1e-3 * (i + 1), device=dev) for i in range(G)]
    e = FusedSAEEnsemble(models, FunctionalSAE, batch_size=B, device=dev)
    x = (torch.randn(B, d, device=dev) * 0.4).to(torch.bfloat16)
    for _ in range(20):
        e.step_batch(x)
    kernels = {
        "enc": lambda: gemm.encode_relu(x, e.enc_shadow, e.params["encoder_bias"], e.c, e.enc_part, None, None,
                                        mask_out=e.cmask),
        "dec": lambda: gemm.decode_residual(e.c, e.dec_shadow, x, e.r, e.dec_part),
        "dc": lambda: gemm.code_grad(e.r, e.dec_shadow, e.c, e.l1, e.dpre, e.colpart, mask=e.cmask),
        "wgrad2": lambda: gemm.weight_grads([[(e.c, e.r)], [(e.dpre, x)]], [e.g_dec, e.g_enc], 1e-6),
    }
    cfgs = {"enc": [1, 5, 9, 13], "dec": [1, 5, 9, 13], "dc": [1, 5, 9, 13], "wgrad2": [3, 7, 11, 15, 1]}
    res = {(k, c): [] for k in kernels for c in cfgs[k]}
    for _ in range(int(os.environ.get("AB_ROUNDS", "7"))):
        for k, fn in kernels.items():
            for c in cfgs[k]:
                with gemm.force_shape(c):
                    res[(k, c)].append(t_once(fn))
    for (k, c), ts in res.items():
        print(json.dumps({"kernel": k, "cfg": c, "shape": gemm.SHAPES[c & 3], "pipe": gemm.PIPES[c >> 2],
                          "median_us": round(statistics.median(ts), 2), "min_us": round(min(ts), 2)}), flush=True)


if __name__ == "__main__":
    main()
