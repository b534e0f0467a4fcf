"""Minimal probe: do back-to-back replays of a HIP graph with a forked side-stream branch keep stream
order on MI355X?  Graph: main x += 1 -> side (waits main): [spin] y = x * 1 -> main waits side: z += y.
With correct ordering z after R replays = sum_{r=1..R} (x0 + r).  Variants: spin on the side branch or
on the main stream, replays back to back or with a host sync between them."""
import json
import torch


def run(spin_side_us, spin_main_us, replays, sync_between, join_end=True):
    dev = torch.device("cuda")
    x = torch.zeros(1, device=dev, dtype=torch.float32)
    y = torch.zeros(1, device=dev, dtype=torch.float32)
    z = torch.zeros(1, device=dev, dtype=torch.float32)
    side = torch.cuda.Stream(dev)
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        cur = torch.cuda.current_stream(dev)
        x.add_(1)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            if spin_side_us:
                torch.cuda._sleep(int(spin_side_us * 2400))
            torch.mul(x, 1, out=y)
        ev = torch.cuda.Event()
        ev.record(side)
        cur.wait_event(ev)
        if spin_main_us:
            torch.cuda._sleep(int(spin_main_us * 2400))
        z.add_(y)
        if join_end:
            cur.wait_stream(side)
    torch.cuda.synchronize()
    for _ in range(replays):
        g.replay()
        if sync_between:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    want = replays * (replays + 1) / 2
    return {"spin_side_us": spin_side_us, "spin_main_us": spin_main_us, "replays": replays,
            "sync_between": sync_between, "z": float(z.item()), "want": want, "ok": float(z.item()) == want}


if __name__ == "__main__":
    for cfg in [(0, 0, 20, False), (200, 0, 20, False), (0, 200, 20, False), (200, 200, 20, False),
                (200, 0, 20, True), (50, 50, 50, False)]:
        print(json.dumps(run(*cfg)), flush=True)
