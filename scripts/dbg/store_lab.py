"""Where does the plain bf16 grouped GEMM spend its time: output stores vs main loop?
Run twice: SC_GEMM_DBG=0 (normal) and SC_GEMM_DBG=1 (EPI_BF16 skips its stores)."""
import json, os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from sparse_coding__amd.ops import gemm


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); s.record()
    for _ in range(iters):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


dev = "cuda"
G, B, n = 8, 2048, 2048
bf = torch.bfloat16
c = torch.empty(G, B, n, device=dev, dtype=bf)
c2 = torch.zeros_like(c)
cases = {"zero_64MB": lambda: c.zero_(), "copy_64MB": lambda: c.copy_(c2)}
for k in (64, 128, 256, 512):
    x = ((torch.rand(B, k, device=dev) * 2 - 1) * 0.5).to(bf)
    w = ((torch.rand(G, n, k, device=dev) * 2 - 1) * 0.05).to(bf)
    for cfg in (1, 3, 9, 13):
        def f(x=x, w=w, cfg=cfg):
            with gemm.force_shape(cfg):
                gemm.matmul_nt(x, w, c)
        cases[f"nt_k{k}_cfg{cfg}"] = f
    cases[f"torch_k{k}"] = lambda x=x, w=w: torch.matmul(x, w.transpose(1, 2), out=c)
res = {k: [] for k in cases}
for _ in range(5):
    for k, f in cases.items():
        try:
            res[k].append(timeit(f))
        except Exception as e:
            res[k].append(float("nan"))
tag = os.environ.get("SC_GEMM_DBG", "0")
for k, v in res.items():
    print(json.dumps({"dbg": tag, "case": k, "median_us": round(statistics.median(v), 2)}), flush=True)
