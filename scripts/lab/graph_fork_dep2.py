"""Probe 5: K consecutive forks (each: torch wait_stream of the side stream on the capturing stream,
then a side op and an event), then the first main node B = A.  Does B keep its dependency on the node
before the forks when K > 1?  Variants re-link the main stream before B."""
import json
import torch


def run(k_forks, relink, replays=12, spin_us=400):
    dev = torch.device("cuda")
    A = torch.zeros(1, device=dev)
    Bh = torch.zeros(replays, device=dev)
    y = torch.zeros(k_forks, device=dev)
    i = torch.zeros(1, dtype=torch.long, device=dev)
    side = torch.cuda.Stream(dev)
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        cur = torch.cuda.current_stream(dev)
        torch.cuda._sleep(int(spin_us * 2400))
        A.add_(1)
        evs = []
        for k in range(k_forks):
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                torch.mul(A, k, out=y[k:k + 1])
            ev = torch.cuda.Event()
            ev.record(side)
            evs.append(ev)
        if relink:
            fence = torch.cuda.Event()
            fence.record(cur)
            cur.wait_event(fence)
        Bh.index_copy_(0, i, A)  # the first main node after the forks
        i.add_(1)
        cur.wait_event(evs[0])
        torch.cuda._sleep(int(spin_us * 2400))
        cur.wait_stream(side)
    torch.cuda.synchronize()
    for _ in range(replays):
        g.replay()
    torch.cuda.synchronize()
    got = Bh.tolist()
    return {"k_forks": k_forks, "relink": relink, "B": got, "ok": got == [float(r + 1) for r in range(replays)]}


if __name__ == "__main__":
    for cfg in [(1, False), (2, False), (5, False), (5, True)]:
        print(json.dumps(run(*cfg)), flush=True)
