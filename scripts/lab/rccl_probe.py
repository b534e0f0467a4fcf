"""RcclComm smoke on one GPU: without a process group, then under a 1-rank nccl process group
(the bench's --force-dist), each with an all-reduce, an all-gather and a captured all-reduce."""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from sparse_coding__amd.parallel.dist import DistInfo, init_distributed  # noqa: E402
from sparse_coding__amd.parallel.rccl import RcclComm  # noqa: E402


def exercise(info, tag):
    print(tag, "init", flush=True)
    c = RcclComm(info)
    print(tag, "comm ok", flush=True)
    t = torch.ones(1024, device=info.device)
    c.all_reduce(t)
    torch.cuda.synchronize()
    print(tag, "all_reduce", float(t.sum()), flush=True)
    o = torch.empty(1024, device=info.device)
    c.all_gather(o, t)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        ev = c.all_reduce(t, overlap=True)
        torch.cuda.current_stream().wait_event(ev)
    g.replay()
    torch.cuda.synchronize()
    print(tag, "captured ok", float(t.sum()), flush=True)
    c.close()
    print(tag, "closed", flush=True)


if __name__ == "__main__":
    exercise(DistInfo(device=torch.device("cuda:0")), "nopg")
    info = init_distributed(force=True)
    print("pg", info, flush=True)
    exercise(info, "pg")
