"""Probe 2: does replay N+1's root node run before replay N's main branch is done when the graph forks
a side branch?  Graph: root x += 1 -> fork side: y = x -> main: spin, wait side, z += x + y (reads the
root's x at its END).  Correct ordering: z = sum_r 2 (x0 + r)."""
import json
import torch


def run(spin_main_us, replays, fork=True, sync_between=False):
    dev = torch.device("cuda")
    x = torch.zeros(1, device=dev)
    y = torch.zeros(1, device=dev)
    z = torch.zeros(1, device=dev)
    side = torch.cuda.Stream(dev)
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        cur = torch.cuda.current_stream(dev)
        x.add_(1)
        if fork:
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                torch.mul(x, 1, out=y)
            ev = torch.cuda.Event()
            ev.record(side)
        else:
            torch.mul(x, 1, out=y)
        torch.cuda._sleep(int(spin_main_us * 2400))
        if fork:
            cur.wait_event(ev)
        z.add_(x + y)
    torch.cuda.synchronize()
    for _ in range(replays):
        g.replay()
        if sync_between:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    want = float(replays * (replays + 1))
    return {"fork": fork, "spin_main_us": spin_main_us, "sync_between": sync_between, "z": float(z.item()),
            "want": want, "ok": float(z.item()) == want}


if __name__ == "__main__":
    for cfg in [(300, 10, True), (300, 10, False), (300, 10, True, True), (2000, 5, True), (20, 50, True)]:
        print(json.dumps(run(*cfg)), flush=True)
