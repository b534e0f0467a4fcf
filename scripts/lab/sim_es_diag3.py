"""ES delayed-comm mismatch: which inter-replay barrier makes consecutive group replays agree."""
import sys, os, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import test_sim_comm_gpu as T
from sparse_coding__amd.engine.graph_plan import count_pattern
from sparse_coding__amd.models.signatures import FunctionalSAE
from sparse_coding__amd.parallel.sim_comm import DelayedSimComm

d, n, B = 512, 1024, 256
GROUPS = tuple(int(g) for g in (sys.argv[1] if len(sys.argv) > 1 else "5,5").split(","))
variants = [("sync-eager", True, False, None), ("capt-none", False, True, None),
            ("capt-devsync", False, True, "dev"), ("capt-streamsync", False, True, "stream"),
            ("capt-hostsleep", False, True, "sleep"), ("capt-none-2", False, True, None),
            ("capt-bsqclean", False, True, "bsq")]
rings = T._rings(d, B, 41, copies=len(variants))
models = [FunctionalSAE.init(d, n, l1, device="cuda") for l1 in (1e-4, 1e-3, 3e-3, 1e-2)]
res = {}
for i, (name, sync, cap, barrier) in enumerate(variants):
    comm = DelayedSimComm("cuda", world=2, delay_us=0, sync=sync)
    ges, es = T._es(models, comm, rings[i], B, d, capture=cap)
    ges.prime([count_pattern(s) for s in sorted(set(GROUPS))])
    dirty = []
    for s in GROUPS:
        dirty.append(bool(es.engine._bsq_dirty))
        if barrier == "bsq":
            es.engine._bsq_dirty = False
        ges.run(s, count_pattern(s))
        if barrier == "dev":
            torch.cuda.synchronize()
        elif barrier == "stream":
            torch.cuda.current_stream().synchronize()
        elif barrier == "sleep":
            time.sleep(0.05)
    torch.cuda.synchronize()
    res[name] = ({k: v.clone() for k, v in es.engine.params.items()}, es.engine.out.clone(), dirty)
ref = res["sync-eager"]
for name, (p, o, dirty) in res.items():
    print(GROUPS, name, "out", float((o - ref[1]).abs().max()),
          "params", max(float((p[k] - ref[0][k]).abs().max()) for k in p), "bsq_dirty before each run", dirty)
