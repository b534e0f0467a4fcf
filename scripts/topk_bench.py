"""Top-k select timing vs torch.topk (config 4 shapes: 8 models x 2048 rows, k = 8..128),
plus the device slot-list build and slot-list weight gradient of the small-k models."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from scripts.kernel_bench import timeit  # noqa: E402


def main():
    from sparse_coding__amd.ops import topk as T

    dev = "cuda"
    ks = [8, 16, 24, 32, 48, 64, 96, 128]
    for n in (6144, 2048):
        scores = torch.randn(8, 2048, n, device=dev)
        k = torch.tensor(ks, dtype=torch.int32, device=dev)
        res = {}
        res["select"] = timeit(lambda: T.topk_select(scores, k, 128), iters=50)
        res["torch_topk_k128"] = timeit(lambda: torch.topk(scores, 128, dim=-1), iters=20)
        idx, val = T.topk_select(scores, k, 128)
        lists = T.SlotLists(3, 2048, n, ks, 128, dev)
        res["slot_lists_k8_16_24"] = timeit(lambda: T.slot_lists(idx, k, lists), iters=50)
        d = 768
        r = torch.randn(8, 2048, d, device=dev).to(torch.bfloat16)
        x = torch.randn(2048, d, device=dev).to(torch.bfloat16)
        g = torch.empty(3, n, d, device=dev, dtype=torch.bfloat16)
        res["sparse_wgrad_k8_16_24_d768"] = timeit(lambda: T.sparse_wgrad(lists, val, val, r, x, g, 1.0), iters=50)
        print(json.dumps({"n": n, **{kk: round(v, 1) for kk, v in res.items()},
                          "read_GBps_select": round(scores.numel() * 4 / res["select"] / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
