"""Process launch and job dispatch on one node.

Reference: ``cluster_runs.py:15-160`` -- one ``mp.Process`` per ensemble sharing a
pinned, shared-memory CPU chunk, ``mp.Value`` done/progress flags polled at 10 Hz,
and a progress bar.  The MI355X design moves the data to HBM (each rank loads its
chunk into its own GPU's ring; no CPU tensor is shared) and uses one process per
GPU, so two pieces remain:

* ``launch(module_or_script, nproc)`` -- a torchrun-style launcher: spawns ``nproc``
  child processes with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set
  (127.0.0.1), streams nothing, returns the exit codes.  It never initialises the GPU
  itself (children own their devices) and never ``exec``s.
* ``dispatch(jobs, devices)`` -- the ``dispatch_job_on_chunk`` analogue for Python
  callables: one spawned worker per device pulls jobs from a queue, reports progress
  through shared counters, and ``monitor`` polls them (the reference's 10 Hz loop).
"""

from __future__ import annotations

import os
import socket
import subprocess
import sys
import time
from typing import Callable, List, Optional, Sequence, Tuple


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(target: str, nproc: int, args: Sequence[str] = (), module: bool = True, env: Optional[dict] = None,
           port: Optional[int] = None, timeout: Optional[float] = None) -> List[int]:
    """Run ``python -m target`` (or ``python target``) as ``nproc`` ranks; returns exit codes."""
    port = port or free_port()
    procs = []
    for r in range(nproc):
        e = dict(os.environ)
        e.update(env or {})
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc), LOCAL_WORLD_SIZE=str(nproc),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        cmd = [sys.executable] + (["-m", target] if module else [target]) + list(args)
        procs.append(subprocess.Popen(cmd, env=e))
    deadline = None if timeout is None else time.time() + timeout
    codes = []
    for p in procs:
        try:
            codes.append(p.wait(timeout=None if deadline is None else max(1.0, deadline - time.time())))
        except subprocess.TimeoutExpired:
            for q in procs:
                if q.poll() is None:
                    q.kill()
            codes.append(-9)
    return codes


def _worker(queue, device, progress, done, results):
    while True:
        item = queue.get()
        if item is None:
            break
        idx, fn, args, kwargs = item
        try:
            results.put((idx, fn(*args, device=device, progress=progress, **kwargs), None))
        except Exception as exc:  # report, keep serving
            results.put((idx, None, repr(exc)))
    done.value = 1


def dispatch(jobs: Sequence[Tuple[Callable, tuple, dict]], devices: Sequence[str], poll: float = 0.1,
             on_progress: Optional[Callable[[int], None]] = None) -> List[Tuple[object, Optional[str]]]:
    """Run ``fn(*args, device=..., progress=..., **kwargs)`` for every job across one worker per
    device.  ``progress`` is a shared ``mp.Value('i')`` the job may increment.  Returns
    ``[(result, error)]`` in job order."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q, res = ctx.Queue(), ctx.Queue()
    for i, (fn, a, kw) in enumerate(jobs):
        q.put((i, fn, a, kw))
    workers, flags, counters = [], [], []
    for dev in devices:
        q.put(None)
        done, prog = ctx.Value("i", 0), ctx.Value("i", 0)
        p = ctx.Process(target=_worker, args=(q, dev, prog, done, res))
        p.start()
        workers.append(p)
        flags.append(done)
        counters.append(prog)
    out: List[Tuple[object, Optional[str]]] = [(None, "not run")] * len(jobs)
    got = 0
    while got < len(jobs):
        try:
            i, r, err = res.get(timeout=poll)
            out[i] = (r, err)
            got += 1
        except Exception:
            if all(f.value for f in flags) and res.empty():
                break
        if on_progress is not None:
            on_progress(sum(c.value for c in counters))
    for p in workers:
        p.join()
    return out


def main(argv=None):
    import argparse

    ap = argparse.ArgumentParser(description="one-node launcher: python -m sparse_coding__amd.train.launch "
                                             "--nproc 8 -m sparse_coding__amd.train.experiments run_single_layer")
    ap.add_argument("--nproc", type=int, default=0, help="ranks (default: number of GPUs)")
    ap.add_argument("-m", "--module", default=None)
    ap.add_argument("script", nargs="?")
    ap.add_argument("rest", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    nproc = a.nproc
    if not nproc:
        import torch

        nproc = max(1, torch.cuda.device_count())  # does not initialise the GPU
    target, module = (a.module, True) if a.module else (a.script, False)
    codes = launch(target, nproc, ([a.script] if a.module and a.script else []) + list(a.rest), module=module)
    return max((abs(c) for c in codes), default=0)


if __name__ == "__main__":
    raise SystemExit(main())
