"""Top-k select timing: wave-bisection kernel vs block-radix kernel vs torch.topk
(config 4 shapes: 8 models x 2048 rows x n = 6144, k = 8..128)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from scripts.kernel_bench import timeit  # noqa: E402


def main():
    from sparse_coding__amd.ops import topk as T

    dev = "cuda"
    for n in (6144, 2048):
        scores = torch.randn(8, 2048, n, device=dev)
        k = torch.tensor([8, 16, 24, 32, 48, 64, 96, 128], dtype=torch.int32, device=dev)
        res = {}
        os.environ.pop("SC_TOPK_RADIX", None)
        res["wave"] = timeit(lambda: T.topk_select(scores, k, 128), iters=50)
        os.environ["SC_TOPK_RADIX"] = "1"
        res["radix"] = timeit(lambda: T.topk_select(scores, k, 128), iters=50)
        os.environ.pop("SC_TOPK_RADIX", None)
        res["torch_topk_k128"] = timeit(lambda: torch.topk(scores, 128, dim=-1), iters=20)
        print(json.dumps({"n": n, **{kk: round(v, 1) for kk, v in res.items()},
                          "read_GBps_wave": round(scores.numel() * 4 / res["wave"] / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
