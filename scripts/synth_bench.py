"""Synthetic activation generation rate (K17): the torch generator vs the Philox code kernel +
MFMA mixing GEMM, bench.py's ring shape (d = 512, 4096 ground-truth features, 32 active on
average, 65536-row batches)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from sparse_coding__amd.data.synthetic import RandomDatasetGenerator

res = {}
for backend in ("torch", "hip"):
    gen = RandomDatasetGenerator(activation_dim=512, n_ground_truth_components=4096, batch_size=65536,
                                 feature_num_nonzero=32, feature_prob_decay=0.999, correlated=False, device="cuda",
                                 seed=1234, backend=backend)
    for _ in range(2):
        gen.send(None)
    torch.cuda.synchronize()
    t = time.perf_counter()
    reps = 10
    for _ in range(reps):
        gen.send(None)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t) / reps
    res[backend] = {"ms_per_batch": round(1e3 * el, 3), "rows_per_s": round(65536 / el, 1),
                    "gb_per_s_bf16": round(65536 * 512 * 2 / el / 1e9, 1)}
print(json.dumps({"what": "synthetic activations, d=512, 4096 features, batch 65536", **res}))
