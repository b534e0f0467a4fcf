"""Probe 6: the lost main-stream dependency after several captured forks -- threshold and fixes."""
import json
import torch


def run(k_forks, variant, replays=12, spin_us=400):
    dev = torch.device("cuda")
    A = torch.zeros(1, device=dev)
    Bh = torch.zeros(replays, device=dev)
    y = torch.zeros(k_forks, device=dev)
    dummy = torch.zeros(1, device=dev)
    i = torch.zeros(1, dtype=torch.long, device=dev)
    side = torch.cuda.Stream(dev)
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        cur = torch.cuda.current_stream(dev)
        torch.cuda._sleep(int(spin_us * 2400))
        A.add_(1)
        evs = []
        shared = None
        if variant == "shared-event":
            shared = torch.cuda.Event()
            shared.record(cur)
        for k in range(k_forks):
            if variant == "fork-once":
                if k == 0:
                    side.wait_stream(cur)
            elif variant == "shared-event":
                side.wait_event(shared)
            else:
                side.wait_stream(cur)
            with torch.cuda.stream(side):
                torch.mul(A, k, out=y[k:k + 1])
            ev = torch.cuda.Event()
            ev.record(side)
            evs.append(ev)
            if variant == "dummy-each":
                dummy.add_(0)
        if variant == "dummy-after":
            dummy.add_(0)
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
    return {"k_forks": k_forks, "variant": variant, "ok": got == [float(r + 1) for r in range(replays)],
            "B": got[:4]}


if __name__ == "__main__":
    for k in (3, 4):
        print(json.dumps(run(k, "plain")), flush=True)
    for v in ("fork-once", "shared-event", "dummy-each", "dummy-after"):
        print(json.dumps(run(5, v)), flush=True)
