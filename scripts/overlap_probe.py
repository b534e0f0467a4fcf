"""Does a memory-bound Adam overlap a GEMM on MI355X?  Times each kernel alone and
the pair on two streams (config 2 shapes): enc || Adam(decoder), wgrad(decoder) ||
Adam(encoder)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from scripts.kernel_bench import timeit  # noqa: E402


def main():
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.models.signatures import FunctionalSAE
    from sparse_coding__amd.ops import adam as adam_ops
    from sparse_coding__amd.ops import gemm

    B, d, n, G = 2048, 512, 2048, 8
    dev = "cuda"
    models = [FunctionalSAE.init(d, n, 1e-3 * (i + 1), device=dev) for i in range(G)]
    e = FusedSAEEnsemble(models, FunctionalSAE, batch_size=B, device=dev)
    x = (torch.randn(B, d, device=dev) * 0.4).to(torch.bfloat16)
    e.step_batch(x)
    sets = e._adam_sets()
    side = torch.cuda.Stream()
    main = torch.cuda.current_stream()

    def enc():
        gemm.encode_relu(x, e.enc_shadow, e.params["encoder_bias"], e.c, e.enc_part, None, None)

    def wdec():
        gemm.weight_grads([[(e.c, e.r)]], [e.g_dec], 1e-6)

    def adam_dec():
        adam_ops.adam_rows(sets[:1], e.lr, 3)

    def adam_enc():
        adam_ops.adam_rows(sets[1:], e.lr, 3)

    def pair(a, b):
        def f():
            side.wait_stream(main)
            with torch.cuda.stream(side):
                b()
            a()
            main.wait_stream(side)
        return f

    def seq(a, b):
        def f():
            a()
            b()
        return f

    res = {"enc": timeit(enc, 100), "adam_dec": timeit(adam_dec, 100), "wgrad_dec": timeit(wdec, 100),
           "adam_enc": timeit(adam_enc, 100)}
    res["enc+adam_dec seq"] = timeit(seq(enc, adam_dec), 100)
    res["enc||adam_dec"] = timeit(pair(enc, adam_dec), 100)
    res["adam_dec||enc (adam first)"] = timeit(pair(adam_dec, enc), 100)
    res["wgrad_dec+adam_enc seq"] = timeit(seq(wdec, adam_enc), 100)
    res["wgrad_dec||adam_enc"] = timeit(pair(wdec, adam_enc), 100)
    print(json.dumps({k: round(v, 1) for k, v in res.items()}))


if __name__ == "__main__":
    main()
