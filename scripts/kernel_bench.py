"""Per-kernel timing of the fused SAE step vs. hipBLASLt (torch.bmm) on the same shapes.

python scripts/kernel_bench.py [--B 2048 --d 512 --n 2048 --G 8]
Prints one JSON line per kernel: time (us), TFLOP/s, and the torch reference time.
"""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def timeit(fn, iters=50, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=2048)
    ap.add_argument("--d", type=int, default=512)
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--G", type=int, default=8)
    a = ap.parse_args()
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.models.signatures import FunctionalSAE
    from sparse_coding__amd.ops import adam as adam_ops
    from sparse_coding__amd.ops import gemm

    dev = "cuda"
    B, d, n, G = a.B, a.d, a.n, a.G
    models = [FunctionalSAE.init(d, n, 1e-3 * (i + 1), device=dev) for i in range(G)]
    e = FusedSAEEnsemble(models, FunctionalSAE, batch_size=B, device=dev)
    x = (torch.randn(B, d, device=dev)).to(torch.bfloat16)
    e.step_batch(x)
    fl = 2.0 * B * n * d * G
    res = {}
    res["enc"] = (timeit(lambda: gemm.encode_relu(x, e.enc_shadow, e.params["encoder_bias"], e.c, e.enc_part,
                                                  e.cnt_part, None)), fl)
    res["dec"] = (timeit(lambda: gemm.decode_residual(e.c, e.dec_shadow, x, e.r, e.dec_part)), fl)
    res["dc"] = (timeit(lambda: gemm.code_grad(e.r, e.dec_shadow, e.c, e.l1, e.dpre, e.colpart, dotpart=e.dotpart)), fl)
    res["wgrad2"] = (timeit(lambda: gemm.weight_grads([[(e.c, e.r)], [(e.dpre, x)]], [e.g_dec, e.g_enc],
                                                      1e-6)), 2 * fl)
    res["enc_nocount"] = (timeit(lambda: gemm.encode_relu(x, e.enc_shadow, e.params["encoder_bias"], e.c,
                                                          e.enc_part, None, None)), fl)
    res["enc_plain_bf16"] = (timeit(lambda: gemm.matmul_nt(x, e.enc_shadow, e.c)), fl)
    res["dc_nodot"] = (timeit(lambda: gemm.code_grad(e.r, e.dec_shadow, e.c, e.l1, e.dpre, e.colpart)), fl)
    res["dc_mask"] = (timeit(lambda: gemm.code_grad(e.r, e.dec_shadow, e.c, e.l1, e.dpre, e.colpart,
                                                    mask=e.cmask)), fl)
    res["enc_mask"] = (timeit(lambda: gemm.encode_relu(x, e.enc_shadow, e.params["encoder_bias"], e.c,
                                                       e.enc_part, None, None, mask_out=e.cmask)), fl)
    res["wgrad_adam"] = (timeit(lambda: e.wgrad_adam(x)), 2 * fl)
    e.overlap_adam = False
    res["step_no_overlap"] = (timeit(lambda: e.step_batch(x)), 5 * fl)
    e.overlap_adam = False
    for cfg in (1, 2, 3):
        for epi in range(7):
            gemm.set_config(epi, cfg)
        res[f"enc_cfg{cfg}"] = (timeit(lambda: gemm.encode_relu(x, e.enc_shadow, e.params["encoder_bias"], e.c,
                                                                e.enc_part, e.cnt_part, None)), fl)
        res[f"dec_cfg{cfg}"] = (timeit(lambda: gemm.decode_residual(e.c, e.dec_shadow, x, e.r, e.dec_part)), fl)
        res[f"dc_cfg{cfg}"] = (timeit(lambda: gemm.code_grad(e.r, e.dec_shadow, e.c, e.l1, e.dpre, e.colpart)), fl)
        res[f"wgrad2_cfg{cfg}"] = (timeit(lambda: gemm.weight_grads([[(e.c, e.r)], [(e.dpre, x)]],
                                                                    [e.g_dec, e.g_enc], 1e-6)), 2 * fl)
        res[f"step_cfg{cfg}"] = (timeit(lambda: e.step_batch(x)), 5 * fl)
    for epi in range(7):
        gemm.set_config(epi, 0)
    res["adam"] = (timeit(lambda: adam_ops.adam_rows(e._adam_sets(), e.lr, 3)), 0)
    res["bias_loss"] = (timeit(lambda: e._bias_loss(True, False)), 0)
    res["step"] = (timeit(lambda: e.step_batch(x)), 5 * fl)
    e.enable_graph()
    e.x_static.copy_(x)
    res["step_graph"] = (timeit(lambda: e.step_static()), 5 * fl)
    e.enable_graph(False)
    # torch / hipBLASLt reference for the same GEMM shapes (bf16 in, bf16 out)
    xe = x.expand(G, B, d)
    we = e.enc_shadow
    ref = {}
    ref["enc"] = timeit(lambda: torch.bmm(xe, we.transpose(1, 2)))
    ref["dec"] = timeit(lambda: torch.bmm(e.c, e.dec_shadow))
    ref["dc"] = timeit(lambda: torch.bmm(e.r, e.dec_shadow.transpose(1, 2)))
    ref["wgrad2"] = timeit(lambda: (torch.bmm(e.c.transpose(1, 2), e.r), torch.bmm(e.dpre.transpose(1, 2), xe)))
    for k, (t, f) in res.items():
        rec = {"kernel": k, "us": round(t, 2), "tflops": round(f / t / 1e6, 1) if f else None,
               "torch_us": round(ref[k], 2) if k in ref else None, "B": B, "d": d, "n": n, "G": G}
        print(json.dumps(rec))


if __name__ == "__main__":
    main()
