"""Probe 3: the graphed ensemble-sharding topology in plain torch ops.  Root R writes slot 0 of s
buffers; a side stream copies slot 0 -> slot 1 of each (one fork per copy, an event after each); the
main stream runs s "steps" (a spin, then it consumes buffer k after waiting event k); replays back to
back.  Correct: every step sees its own replay's data."""
import json
import torch


def run(s=5, replays=4, spin_us=300, variant="es", sync_between=False):
    dev = torch.device("cuda")
    counter = torch.zeros(1, device=dev)
    glob = torch.zeros(s, 2, device=dev)
    seen = torch.zeros(replays * s, 2, device=dev)
    idx = torch.zeros(1, dtype=torch.long, device=dev)
    side = torch.cuda.Stream(dev)
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        cur = torch.cuda.current_stream(dev)
        # root: slot 0 of every buffer = the replay's value (counter + 1 + k)
        counter.add_(1)
        glob[:, 0].copy_(counter * 100 + torch.arange(s, device=dev, dtype=torch.float32))
        evs = []
        for k in range(s):
            if variant != "fork-once" or k == 0:
                side.wait_stream(cur)
            with torch.cuda.stream(side):
                torch.mul(glob[k, 0:1], 1, out=glob[k, 1:2])
            ev = torch.cuda.Event()
            ev.record(side)
            evs.append(ev)
        if variant == "join-first":
            cur.wait_stream(side)
        for k in range(s):
            torch.cuda._sleep(int(spin_us * 2400))
            cur.wait_event(evs[k])
            seen.index_copy_(0, idx, glob[k:k + 1])
            idx.add_(1)
        cur.wait_stream(side)
    torch.cuda.synchronize()
    for _ in range(replays):
        g.replay()
        if sync_between:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    want = torch.tensor([[r * 100 + k] * 2 for r in range(1, replays + 1) for k in range(s)], device=dev,
                        dtype=torch.float32)
    bad = int((seen != want).any(dim=1).sum())
    return {"variant": variant, "s": s, "spin_us": spin_us, "sync_between": sync_between, "bad_steps": bad,
            "of": replays * s, "first_bad": seen[(seen != want).any(dim=1)][:2].tolist()}


if __name__ == "__main__":
    for cfg in [dict(), dict(sync_between=True), dict(variant="fork-once"), dict(variant="join-first"),
                dict(s=3), dict(spin_us=20), dict(spin_us=1000, replays=3)]:
        print(json.dumps(run(**cfg)), flush=True)
