"""Diagnose the ES delayed-comm mismatch: run the graphed ES step in four modes and compare."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import torch
import test_sim_comm_gpu as T
from sparse_coding__amd.models.signatures import FunctionalSAE
from sparse_coding__amd.parallel.sim_comm import DelayedSimComm

d, n, B = 512, 1024, 256
GROUPS = tuple(int(g) for g in (sys.argv[1] if len(sys.argv) > 1 else "3,5,3").split(","))
rings = T._rings(d, B, 41, copies=5)
models = [FunctionalSAE.init(d, n, l1, device="cuda") for l1 in (1e-4, 1e-3, 3e-3, 1e-2)]
runs = {}
for i, (name, kw, cap) in enumerate([("sync-eager", dict(delay_us=0, sync=True), False),
                                     ("sync-capt", dict(delay_us=0, sync=True), True),
                                     ("delay-eager", dict(delay_us=50), False),
                                     ("delay0-capt", dict(delay_us=0), True),
                                     ("delay-capt", dict(delay_us=50), True)]):
    ges, es = T._es(models, DelayedSimComm("cuda", world=2, **kw), rings[i], B, d, capture=cap)
    T._run_es(ges, GROUPS)
    runs[name] = (ges, es)
ref = runs["sync-eager"][1].engine
for name, (ges, es) in runs.items():
    e = es.engine
    diffs = {k: float((e.params[k] - ref.params[k]).abs().max()) for k in e.params}
    print(GROUPS, name, "out", float((e.out - ref.out).abs().max()), diffs,
          "glob", float((ges._glob.float() - runs["sync-eager"][0]._glob.float()).abs().max()),
          "step", int(e.step_dev.item()))
