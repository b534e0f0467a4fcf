"""ES mismatch: per-step history (the batch each step trained on, its losses) captured inside the graph."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import test_sim_comm_gpu as T
from sparse_coding__amd.engine.fused import FusedSAEEnsemble
from sparse_coding__amd.engine.graph_plan import count_pattern
from sparse_coding__amd.models.signatures import FunctionalSAE
from sparse_coding__amd.parallel.sim_comm import DelayedSimComm

d, n, B = 512, 1024, 256
GROUPS = (5, 5)
TOTAL = sum(GROUPS)
HIST = {}
orig = FusedSAEEnsemble._step_kernels


def hooked(self, x, count=None, gather=None, before_update=None):
    h = HIST[id(self)]
    # before the step: the batch it trains on and the step counter it sees
    h["x"].index_copy_(0, h["slot"], x.unsqueeze(0)) if False else None
    torch.index_select(self.step_dev.long(), 0, torch.zeros(1, dtype=torch.long, device=x.device), out=h["tmp"])
    h["steps"].index_copy_(0, h["tmp"], self.step_dev.float())
    h["xs"].index_copy_(0, h["tmp"], x.float().sum(dim=1, keepdim=True).t())
    orig(self, x, count, gather, before_update)
    h["outs"].index_copy_(0, h["tmp"], self.out[:, 0].unsqueeze(0))


FusedSAEEnsemble._step_kernels = hooked

res = {}
rings = T._rings(d, B, 41, copies=3)
models = [FunctionalSAE.init(d, n, l1, device="cuda") for l1 in (1e-4, 1e-3, 3e-3, 1e-2)]
for i, (name, sync, cap, between) in enumerate([("ref", True, False, False), ("capt", False, True, False),
                                                 ("capt-sync", False, True, True)]):
    ges, es = T._es(models, DelayedSimComm("cuda", world=2, delay_us=0, sync=sync), rings[i], B, d, capture=cap)
    e = es.engine
    HIST[id(e)] = {"steps": torch.full((TOTAL + 2,), -1.0, device="cuda"), "tmp": torch.zeros(1, dtype=torch.long, device="cuda"),
                   "xs": torch.zeros(TOTAL + 2, 2 * B, device="cuda"), "outs": torch.zeros(TOTAL + 2, 2, device="cuda")}
    ges.prime([count_pattern(s) for s in sorted(set(GROUPS))])
    for s in GROUPS:
        ges.run(s, count_pattern(s))
        if between:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    res[name] = {k: v.clone() for k, v in HIST[id(e)].items() if k != "tmp"}
r = res["ref"]
for name, h in res.items():
    print(name, "steps seen", h["steps"][:TOTAL].tolist())
    for t in range(TOTAL):
        dx = float((h["xs"][t] - r["xs"][t]).abs().max())
        do = float((h["outs"][t] - r["outs"][t]).abs().max())
        print(f"  step {t}: batch diff {dx:.4g}  loss diff {do:.4g}")
