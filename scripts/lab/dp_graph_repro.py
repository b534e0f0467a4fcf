"""Stage-by-stage rehearsal of bench.py's graphed data-parallel runner under a one-rank RCCL group,
with a printed marker and an explicit gc.collect() after every stage (bench.py --force-dist
--parallelism dp --dp-graph 1 segfaulted in GraphedDataParallel.__init__ on the builder box).
Usage: python dp_graph_repro.py [dp|zero1] [order: engines-first|comm-first] [gc: on|off]"""
import faulthandler
import gc
import sys
from pathlib import Path

faulthandler.enable()
sys.path.insert(0, str(Path(__file__).resolve().parents[2]))


def mark(msg):
    print("STAGE", msg, flush=True)


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "dp"
    order = sys.argv[2] if len(sys.argv) > 2 else "engines-first"
    use_gc = (sys.argv[3] if len(sys.argv) > 3 else "on") == "on"
    if not use_gc:
        gc.disable()
    import numpy as np
    import torch

    import bench
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.engine.graph_plan import count_pattern
    from sparse_coding__amd.models.signatures import FunctionalSAE
    from sparse_coding__amd.parallel.dist import init_distributed
    from sparse_coding__amd.parallel.graphed import GraphedDataParallel
    from sparse_coding__amd.parallel.rccl import RcclComm

    def collect(tag):
        if use_gc:
            mark(f"{tag}: gc.collect -> {gc.collect()}")

    info = init_distributed(force=True)
    mark(f"pg {info}")
    collect("pg")
    args = bench.parse(["--force-dist", "--parallelism", mode, "--dp-graph", "1", "--steps", "16", "--warmup", "8"])
    models = [FunctionalSAE.init(512, 2048, float(l1), device=info.device) for l1 in np.logspace(-4, -2, 8)]
    ring, _ = bench.build_ring(args, info.device)
    mark("ring")
    collect("ring")
    comm = None
    if order == "comm-first":
        comm = RcclComm(info)
        mark("comm")
        collect("comm")
    engines = [FusedSAEEnsemble(models, FunctionalSAE, lr=1e-3, batch_size=2048, device=info.device)]
    mark("engines")
    collect("engines")
    if comm is None:
        comm = RcclComm(info)
        mark("comm")
        collect("comm")
    src = ring.graph_source(2048, info.rank, info.world_size)
    mark("source")
    collect("source")
    gdp = GraphedDataParallel(engines, info, comm, src, mode=mode,
                              grad_dtype=torch.bfloat16 if mode == "zero1" else torch.float32)
    mark("gdp")
    collect("gdp")
    gdp.prime([count_pattern(8, 8)])
    mark("primed")
    for _ in range(4):
        gdp.run(8, count_pattern(8, 8))
    torch.cuda.synchronize()
    mark(f"ran: loss {engines[0].out[:, 0].tolist()}")
    comm.close()
    mark("closed")


if __name__ == "__main__":
    main()
