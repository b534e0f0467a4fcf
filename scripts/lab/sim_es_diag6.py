"""ES replay race: keep the captured events alive / add a sink kernel after the join."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import test_sim_comm_gpu as T
from sparse_coding__amd.engine.graph_plan import count_pattern
from sparse_coding__amd.models.signatures import FunctionalSAE
from sparse_coding__amd.parallel import graphed
from sparse_coding__amd.parallel.sim_comm import DelayedSimComm

MODE = {"v": "as-is"}
KEEP = []


def _steps(self, pattern):
    e = self.engine
    s = len(pattern)
    glob = self._buffers(s)[:s]
    self.source.gather_into_global(glob, e.step_dev)
    B, r = self.B, self.es.info.rank
    evs = [self.comm.all_gather(glob[k], glob[k][r * B:(r + 1) * B], overlap=True) for k in range(s)]
    if "keep" in MODE["v"]:
        KEEP.append(evs)
    cur = torch.cuda.current_stream(self.device)
    tail = bool(e._tail_ok)
    if tail:
        self._ep0.copy_(e.step_dev)
        flat = self._glob.view(-1, self.es.d)
    for k, count in enumerate(pattern):
        if k == 0 or not tail:
            if evs[k] is not None:
                cur.wait_event(evs[k])
            self._x.copy_(glob[k])
        nxt = tail and k + 1 < s
        wait = (lambda ev=evs[k + 1]: cur.wait_event(ev)) if nxt and evs[k + 1] is not None else None
        e._counted = count
        e._step_kernels(self._x, count, gather=(flat, self._ident, self._ep0, self._x) if nxt else None,
                        before_update=wait)
    self.comm.join()
    if "sink" in MODE["v"]:
        self._ep0.add_(0)  # a node after the join: the graph's single sink


graphed.GraphedEnsembleSharded._steps = _steps

d, n, B = 512, 1024, 256
GROUPS = (5, 5)
variants = ["ref", "as-is", "keep", "sink", "keep+sink"]
rings = T._rings(d, B, 41, copies=len(variants))
models = [FunctionalSAE.init(d, n, l1, device="cuda") for l1 in (1e-4, 1e-3, 3e-3, 1e-2)]
res = {}
for i, v in enumerate(variants):
    MODE["v"] = v
    ref = v == "ref"
    ges, es = T._es(models, DelayedSimComm("cuda", world=2, delay_us=0, sync=ref), rings[i], B, d, capture=not ref)
    ges.prime([count_pattern(s) for s in sorted(set(GROUPS))])
    for s in GROUPS:
        ges.run(s, count_pattern(s))
    torch.cuda.synchronize()
    res[v] = ({k: t.clone() for k, t in es.engine.params.items()}, es.engine.out.clone())
for v, (p, o) in res.items():
    print(v, "out", float((o - res["ref"][1]).abs().max()),
          "params", max(float((p[k] - res["ref"][0][k]).abs().max()) for k in p), flush=True)
