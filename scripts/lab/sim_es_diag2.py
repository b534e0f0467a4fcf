"""ES delayed-comm mismatch, finer: per-group comparisons and variants of the replay."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import test_sim_comm_gpu as T
from sparse_coding__amd.engine.graph_plan import count_pattern
from sparse_coding__amd.models.signatures import FunctionalSAE
from sparse_coding__amd.parallel.sim_comm import DelayedSimComm


class NoOverlap(DelayedSimComm):
    def all_gather(self, out, inp, overlap=False):
        return super().all_gather(out, inp, overlap=False)


d, n, B = 512, 1024, 256
GROUPS = (5, 5)
variants = [("sync-eager", lambda: DelayedSimComm("cuda", world=2, delay_us=0, sync=True), False, {}),
            ("delay0-capt", lambda: DelayedSimComm("cuda", world=2, delay_us=0), True, {}),
            ("delay0-capt-fresh", lambda: DelayedSimComm("cuda", world=2, delay_us=0), True, {"fresh": 1}),
            ("delay0-capt-sync", lambda: DelayedSimComm("cuda", world=2, delay_us=0), True, {"sync": 1}),
            ("nooverlap-capt", lambda: NoOverlap("cuda", world=2, delay_us=0), True, {}),
            ("delay0-capt-noupload", lambda: DelayedSimComm("cuda", world=2, delay_us=0), True, {"noupload": 1})]
rings = T._rings(d, B, 41, copies=len(variants))
models = [FunctionalSAE.init(d, n, l1, device="cuda") for l1 in (1e-4, 1e-3, 3e-3, 1e-2)]
res = {}
for i, (name, mk, cap, opt) in enumerate(variants):
    ges, es = T._es(models, mk(), rings[i], B, d, capture=cap)
    if opt.get("noupload"):
        from sparse_coding__amd.ops import _lib
        _lib.upload_graph = lambda g, dev: None
    ges.prime([count_pattern(s) for s in sorted(set(GROUPS))])
    snaps = []
    for s in GROUPS:
        if opt.get("fresh"):
            ges._graphs = {}
        ges.run(s, count_pattern(s))
        torch.cuda.synchronize()
        snaps.append((es.engine.out.clone(), {k: v.clone() for k, v in es.engine.params.items()},
                      ges._glob.clone(), ges._x.clone()))
    res[name] = snaps
ref = res["sync-eager"]
for name, snaps in res.items():
    for gi, (o, p, g, x) in enumerate(snaps):
        ro, rp, rg, rx = ref[gi]
        print(name, "group", gi, "out", float((o - ro).abs().max()),
              "params", max(float((p[k] - rp[k]).abs().max()) for k in p),
              "glob", float((g.float() - rg.float()).abs().max()), "x", float((x.float() - rx.float()).abs().max()))
