"""Probe 4: does the first main-stream node captured after a fork (event recorded on the capturing
stream, waited by a side stream) keep its dependency on the node before the fork?  Graph:
A += 1 -> fork (side: y = A) -> B = A -> main spin -> z += B (and join).  B must equal A of the same
replay.  Variants: plain fork (torch wait_stream), fork + the main stream re-waiting the fork event."""
import json
import torch


def run(variant, replays=12, spin_us=400):
    dev = torch.device("cuda")
    A = torch.zeros(1, device=dev)
    Bh = torch.zeros(replays, device=dev)
    y = torch.zeros(1, device=dev)
    i = torch.zeros(1, dtype=torch.long, device=dev)
    side = torch.cuda.Stream(dev)
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        cur = torch.cuda.current_stream(dev)
        torch.cuda._sleep(int(spin_us * 2400))   # long tail of the previous replay ... then
        A.add_(1)
        if variant == "wait_stream":
            side.wait_stream(cur)
        else:
            ev = torch.cuda.Event()
            ev.record(cur)
            side.wait_event(ev)
            if variant == "rewait":
                cur.wait_event(ev)
        with torch.cuda.stream(side):
            torch.mul(A, 1, out=y)
        Bh.index_copy_(0, i, A)  # the first main node after the fork
        i.add_(1)
        torch.cuda._sleep(int(spin_us * 2400))
        cur.wait_stream(side)
    torch.cuda.synchronize()
    for _ in range(replays):
        g.replay()
    torch.cuda.synchronize()
    got = Bh.tolist()
    want = [float(r + 1) for r in range(replays)]
    return {"variant": variant, "B": got, "ok": got == want}


if __name__ == "__main__":
    for v in ("wait_stream", "event", "rewait"):
        print(json.dumps(run(v)), flush=True)
