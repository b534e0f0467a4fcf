"""``HostComm`` (parallel/host_comm.py): the RcclComm interface over gloo, checked on CPU tensors with
3 ranks -- every collective the graphed multi-GPU steps use, in place and with bf16 payloads."""

import os
import socket

import numpy as np
import torch
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from sparse_coding__amd.parallel.dist import DistInfo
    from sparse_coding__amd.parallel.host_comm import HostComm

    dist.init_process_group("gloo", rank=rank, world_size=world)
    c = HostComm(DistInfo(rank, world, rank, torch.device("cpu"), "gloo"))
    out = {}
    t = torch.arange(12, dtype=torch.float32) * (rank + 1)
    c.all_reduce(t)
    out["all_reduce"] = t.numpy()
    tb = (torch.arange(12, dtype=torch.float32) * 0.5 * (rank + 1)).to(torch.bfloat16)
    c.all_reduce(tb)
    out["all_reduce_bf16"] = tb.float().numpy()
    inp = torch.arange(12, dtype=torch.float32) + 100 * rank
    rs = torch.empty(4)
    c.reduce_scatter(rs, inp)
    out["reduce_scatter"] = rs.numpy()
    g = torch.zeros(world, 5, dtype=torch.bfloat16)
    g[rank] = torch.full((5,), float(rank + 1))
    c.all_gather(g.view(-1), g[rank])  # in place: this rank's block of the output
    out["all_gather"] = g.float().numpy()
    a2a_in = (torch.arange(world * 2, dtype=torch.float32) + 10 * rank).to(torch.bfloat16)
    a2a_out = torch.empty_like(a2a_in)
    c.all_to_all(a2a_out, a2a_in)
    out["all_to_all"] = a2a_out.float().numpy()
    b = torch.full((3,), float(rank))
    c.broadcast(b, root=1)
    out["broadcast"] = b.numpy()
    out["calls"] = dict(c.calls)
    q.put((rank, out))
    dist.destroy_process_group()


def test_host_comm_collectives_three_ranks():
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    base = np.arange(12, dtype=np.float32)
    for r in range(world):
        o = res[r]
        np.testing.assert_array_equal(o["all_reduce"], base * 6)
        np.testing.assert_allclose(o["all_reduce_bf16"], base * 0.5 * 6, rtol=1e-2)
        total = sum(base + 100 * rr for rr in range(world))
        np.testing.assert_array_equal(o["reduce_scatter"], total[4 * r:4 * r + 4])
        np.testing.assert_array_equal(o["all_gather"], np.repeat(np.arange(1, world + 1, dtype=np.float32)[:, None], 5, 1))
        # out block j = rank j's input block r
        want = np.concatenate([(np.arange(world * 2, dtype=np.float32) + 10 * j)[2 * r:2 * r + 2] for j in range(world)])
        np.testing.assert_array_equal(o["all_to_all"], want)
        np.testing.assert_array_equal(o["broadcast"], np.ones(3))
        assert o["calls"] == {"all_reduce": 2, "reduce_scatter": 1, "all_gather": 1, "all_to_all": 1, "broadcast": 1}
