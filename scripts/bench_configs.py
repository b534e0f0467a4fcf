"""Throughput of the other BASELINE.json configs (bench.py covers config 2 / 3).

  python scripts/bench_configs.py cpu      # config 1: tied SAE d=128 ratio 2 l1=1e-3, CPU eager
  python scripts/bench_configs.py topk     # config 4: GPT-2-small residual (d=768), ratio 8, top-k
  python scripts/bench_configs.py fista    # config 5: FISTA 300-step dictionary learning, d=1024
  python scripts/bench_configs.py mlpout   # config 3: Pythia-70m MLP-out (hook_mlp_out, d=512), DP path
  python scripts/bench_configs.py mlp      # Pythia-70m MLP hidden (hook_post, d_mlp=2048) shapes

Every line is one JSON record: activations/s over the timed steps (full steps: gather,
forward, backward, optimiser, and for FISTA the solve + basis update), synthetic data,
random-init weights.
"""

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch


def _timed(step, steps, warmup, sync):
    for _ in range(warmup):
        step()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    return time.perf_counter() - t0


def _ring(d, device, rows=1 << 19, feats=None, k=32, gb=0.0):
    """HBM ring of synthetic rows; ``gb`` > 0 sizes it in GB of device memory instead (the
    288 GB MI355X holds ~130 M rows of d = 1024 bf16 in a 270 GB ring)."""
    from sparse_coding__amd.data.ring import DeviceRing, rows_for_budget
    from sparse_coding__amd.data.synthetic import RandomDatasetGenerator

    gen = RandomDatasetGenerator(d, feats or 8 * d, 65536, k, 0.999, False, device, seed=7)
    dt = torch.bfloat16 if device != "cpu" else torch.float32
    if gb > 0:
        rows = rows_for_budget(d, int(gb * 1e9), dt)
    ring = DeviceRing(rows, d, device=device, dtype=dt, seed=1)
    scale = 9.0 / float(gen.send(None).norm(dim=-1).mean())  # bench.py --act-norm calibration
    ring.fill(lambda: gen.send(None) * scale)
    return ring


def cfg_cpu(a):
    from sparse_coding__amd.engine.trainer import EnsembleTrainer
    from sparse_coding__amd.models.signatures import FunctionalTiedSAE

    torch.manual_seed(0)
    B = 256
    models = [FunctionalTiedSAE.init(128, 256, 1e-3)]
    tr = EnsembleTrainer(models, FunctionalTiedSAE, batch_size=B, device="cpu")
    ring = _ring(128, "cpu", rows=1 << 16)
    el = _timed(lambda: tr.step(ring.sample(B)), a.steps, a.warmup, lambda: None)
    return {"config": "1: tied SAE d=128 ratio 2 l1=1e-3, CPU closed-form engine (reference row 10: 82.9k act/s)",
            "value": round(B * a.steps / el, 1), "unit": "activations/s", "ms_per_step": round(1e3 * el / a.steps, 3),
            "batch": B, "threads": torch.get_num_threads()}


def cfg_topk(a):
    from sparse_coding__amd.engine.topk import FusedTopKEnsemble
    from sparse_coding__amd.models.topk import TopKEncoder

    dev = "cuda:0"
    torch.manual_seed(0)
    d, ratio, B = 768, 8, a.batch
    n = d * ratio
    ks = [8, 16, 24, 32, 48, 64, 96, 128][: a.models]
    models = [TopKEncoder.init(d, n, k, device=dev) for k in ks]
    sk = a.sparse_k if a.sparse_k == "auto" else int(a.sparse_k)
    eng = FusedTopKEnsemble(models, lr=1e-3, batch_size=B, device=dev, sparse_k=sk)
    eng.enable_graph(not a.eager)
    ring = _ring(d, dev)
    gs = max(1, int(a.graph_steps)) if not a.eager else 1
    if gs > 1:  # multi-step graphs with the batch gather inside (engine/topk.py run_source)
        src = ring.graph_source(B)
        steps = max(1, a.steps // gs) * gs
        el = _timed(lambda: eng.run_source(src, gs), steps // gs, max(1, a.warmup // gs), torch.cuda.synchronize)
    else:
        steps = a.steps
        el = _timed(lambda: eng.step_batch(ring.sample(B, out=eng.x_static)), steps, a.warmup, torch.cuda.synchronize)
    return {"config": f"4: GPT-2-small residual d={d}, ratio {ratio} (n={n}), fused top-k, k={ks}",
            "value": round(B * steps / el, 1), "unit": "activations/s", "ms_per_step": round(1e3 * el / steps, 3),
            "steps": steps, "batch": B, "models": len(ks), "sparse_wgrad_models": eng.sparse_g, "graph": not a.eager,
            "graph_steps": gs, "dtype": "bf16", "data": "synthetic"}


def cfg_fista(a):
    from sparse_coding__amd.engine.trainer import EnsembleTrainer
    from sparse_coding__amd.models.fista import FunctionalFista

    dev = "cuda:0"
    torch.manual_seed(0)
    d, ratio, B = 1024, a.ratio, a.batch
    n = int(d * ratio)
    l1s = np.logspace(-4, -2, a.models)
    models = [FunctionalFista.init(d, n, float(l1), device=dev) for l1 in l1s]
    tr = EnsembleTrainer(models, FunctionalFista, batch_size=B, device=dev, fista_iters=a.iters,
                         fista_backend="hip")
    t0 = time.perf_counter()
    ring = _ring(d, dev, gb=a.ring_gb)
    fill_s = time.perf_counter() - t0
    xbuf = torch.empty(B, d, device=dev, dtype=torch.bfloat16)
    el = _timed(lambda: tr.step(ring.sample(B, out=xbuf)), a.steps, a.warmup, torch.cuda.synchronize)
    # FISTA solve alone
    from sparse_coding__amd.ops import fista as F

    D = torch.nn.functional.normalize(torch.randn(a.models, n, d, device=dev), dim=-1)
    x = ring.sample(B).float()
    eta = F.step_size(D)
    lam = torch.tensor(l1s, device=dev, dtype=torch.float32)
    solves = {}
    for form in ("direct", "gram"):
        if form == "gram" and n not in F.GRAM_N:
            continue
        solves[form] = _timed(lambda: F.fista(x, D, lam, None, a.iters, eta, backend="hip", with_res=False,
                                              form=form), 3, 1, torch.cuda.synchronize) / 3
    el_solve = min(solves.values())
    return {"config": f"5: FISTA {a.iters}-step dictionary learning, Pythia-410m-shaped d={d}, n={n}, "
                      f"{a.models} models (reference row 13: 452 ms per model-solve, d=n=512, 500 it, B=256, CPU)",
            "value": round(B * a.steps / el, 1), "unit": "activations/s", "ms_per_step": round(1e3 * el / a.steps, 3),
            "solve_ms_all_models": round(1e3 * el_solve, 3),
            "solve_ms_per_model": round(1e3 * el_solve / a.models, 3),
            "solve_ms_by_form": {k: round(1e3 * v, 3) for k, v in solves.items()},
            "batch": B, "engine": tr.kind, "ring_rows": ring.capacity,
            "ring_gb": round(ring.capacity * d * 2 / 1e9, 1), "ring_fill_s": round(fill_s, 1)}


def cfg_config5(a):
    """Config 5 at machine scale (reference activation_dataset.py:326-391 harvest, big_sweep.py:176-198
    + basic_l1_sweep.py:48-152 training): random-init Pythia-410m in bf16, layer-12 residual
    (d = 1024) harvested into an HBM ring sized from free device memory (all but ``--reserve-gb``),
    then the fork's loop -- ``EnsembleTrainer(..., FunctionalFista)``: one Adam step of the
    8-model L1 sweep, then a 300-iteration FISTA solve + Hessian-preconditioned basis update per
    step, all on device.  Progress lines go to stderr while the ring fills."""
    from sparse_coding__amd.data.harvest import ActivationHarvester, build_model
    from sparse_coding__amd.data.ring import DeviceRing, rows_for_budget
    from sparse_coding__amd.engine.trainer import EnsembleTrainer
    from sparse_coding__amd.models.fista import FunctionalFista
    from sparse_coding__amd.ops import fista as F

    dev = "cuda:0"
    torch.manual_seed(0)
    d, layer = 1024, 12
    model = build_model("pythia-410m", device=dev, dtype=torch.bfloat16)
    h = ActivationHarvester(model, [layer], "residual")
    bs, seq = 64, 256
    free, total = torch.cuda.mem_get_info()
    budget = (a.ring_gb * 1e9) if a.ring_gb > 0 else free - a.reserve_gb * 1e9
    ring = DeviceRing(rows_for_budget(d, int(budget)), d, device=dev, seed=1)
    # Zipf token ids sampled on the device (offline stand-in for the Pile)
    ranks = torch.arange(1, 50305, device=dev, dtype=torch.float64)
    probs = (1.0 / ranks ** 1.1)
    probs = (probs / probs.sum()).float()
    gen = torch.Generator(device=dev).manual_seed(3)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    last = t0
    while ring.size < ring.capacity:
        toks = torch.multinomial(probs, bs * seq, replacement=True, generator=gen).view(bs, seq)
        acts = h.run(toks)[layer]
        ring.push(acts[: ring.capacity - ring.size])
        if time.perf_counter() - last > 20:
            torch.cuda.synchronize()
            last = time.perf_counter()
            print(f"[config5] ring {ring.size / ring.capacity:6.1%} of {ring.capacity} rows, "
                  f"{ring.size / (last - t0):,.0f} act/s", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    fill_s = time.perf_counter() - t0
    h.close()
    del model, h
    torch.cuda.empty_cache()
    B, n = a.batch, int(d * a.ratio)
    l1s = np.logspace(-4, -2, a.models)
    models = [FunctionalFista.init(d, n, float(l1), device=dev) for l1 in l1s]
    tr = EnsembleTrainer(models, FunctionalFista, batch_size=B, device=dev, fista_iters=a.iters, fista_backend="hip")
    xbuf = torch.empty(B, d, device=dev, dtype=torch.bfloat16)
    el = _timed(lambda: tr.step(ring.sample(B, out=xbuf)), a.steps, a.warmup, torch.cuda.synchronize)
    D = torch.nn.functional.normalize(torch.randn(a.models, n, d, device=dev), dim=-1)
    x = ring.sample(B).float()
    eta = F.step_size(D)
    lam = torch.tensor(l1s, device=dev, dtype=torch.float32)
    solve = _timed(lambda: F.fista(x, D, lam, None, a.iters, eta, backend="hip", with_res=False), 3, 1,
                   torch.cuda.synchronize) / 3
    return {"config": f"5: FISTA {a.iters}-step dictionary learning on harvested random-init Pythia-410m layer-{layer} "
                      f"residual (d={d}), n={n}, {a.models} models, batch {B}",
            "value": round(B * a.steps / el, 1), "unit": "activations/s", "ms_per_step": round(1e3 * el / a.steps, 3),
            "solve_ms_all_models": round(1e3 * solve, 3), "engine": tr.kind,
            "ring_rows": ring.capacity, "ring_gb": round(ring.capacity * d * 2 / 1e9, 1),
            "device_total_gb": round(total / 1e9, 1), "ring_fill_s": round(fill_s, 1),
            "harvest_act_per_s": round(ring.capacity / fill_s, 1), "dtype": "bf16", "data": "harvested (random-init LM)"}


def cfg_fistaloss(a):
    """FISTA in the loss (reference autoencoders/fista.py:141-172, the fork's fista_13_10 runs):
    8-model L1 sweep, d = n = 512 (dict_size 512), 50 unrolled iterations inside the loss.
    The fused engine (tied SAE kernels + Gram-form solve / adjoint + row Adam) and, for
    comparison, the autograd engine (HIP solve + adjoint, torch SAE half and Adam)."""
    from sparse_coding__amd.engine.fista_loss import FistaLossEnsemble, FusedFistaLossEnsemble
    from sparse_coding__amd.models.fista import FunctionalFista

    dev = "cuda:0"
    torch.manual_seed(0)
    d, n, B = 512, int(512 * a.ratio), a.batch
    models = [FunctionalFista.init(d, n, float(l1), device=dev) for l1 in np.logspace(-4, -2, a.models)]
    ring = _ring(d, dev)
    xbuf = torch.empty(B, d, device=dev, dtype=torch.bfloat16)
    out = {"config": f"FISTA-in-loss ensemble: d={d}, n={n}, {a.models} models, {a.iters} unrolled iterations",
           "unit": "activations/s", "batch": B, "dtype": "bf16 GEMM operands, fp32 iterates", "data": "synthetic"}
    for name, cls, kw in (("fused", FusedFistaLossEnsemble, {}), ("autograd", FistaLossEnsemble, {"backend": "hip"})):
        eng = cls(models, lr=1e-3, batch_size=B, device=dev, num_iter=a.iters, **kw)
        losses = []
        el = _timed(lambda: losses.append(eng.step_batch(ring.sample(B, out=xbuf))), a.steps, a.warmup,
                    torch.cuda.synchronize)
        out[f"{name}_ms_per_step"] = round(1e3 * el / a.steps, 3)
        out[f"{name}_loss_first"] = [round(float(v), 5) for v in losses[0]]
        out[f"{name}_loss_last"] = [round(float(v), 5) for v in losses[-1]]
        del eng
        torch.cuda.empty_cache()
    out["ms_per_step"] = out["fused_ms_per_step"]
    out["value"] = round(B / out["fused_ms_per_step"] * 1e3, 1)
    return out


def cfg_mlpout(a):
    """Config 3: Pythia-70m MLP-out -- the reference's ``mlpout`` hook is ``hook_mlp_out``, d_model
    = 512 wide (reference activation_dataset.py:66-67, 104-105) -- 8-model L1 sweep, ratio 4, on
    the data-parallel path (BASELINE config 3's mechanism): ``bench.py --parallelism dp``, i.e.
    ChunkedDataParallel over the fused engine with the chunk-pipelined RCCL gradient all-reduce.
    On one GPU it runs under a 1-rank RCCL process group (the collectives are issued but move
    nothing); the N-GPU numbers come from the driver's ``bench.py --parallelism dp`` runs."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--parallelism", "dp", "--force-dist", "--no-eval",
           "--compare-parallelism", "0", "--steps", str(a.steps), "--warmup", str(a.warmup)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise RuntimeError(r.stderr[-2000:])
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    G, n, d = 8, 2048, 512
    grad_bytes = (2 * G * n * d + G * n) * 4
    return {"config": "3: Pythia-70m MLP-out (hook_mlp_out, d=512), ratio 4, 8 models, data-parallel fused step "
                      "(ChunkedDataParallel, 1-rank RCCL group on one GPU)", "unit": "activations/s",
            "value": rec["value"], "ms_per_step": rec["ms_per_step"], "dtype": "bf16", "data": "synthetic",
            "parallelism": rec["config"]["parallelism"], "dp_chunks": rec["config"]["dp_chunks"],
            "allreduce_bytes_per_step": grad_bytes,
            "allreduce_ring_bytes_sent_per_gpu_at_8": round(2 * 7 / 8 * grad_bytes),
            "note": "per-GPU compute of the DP step; the all-reduce is measured by the driver's multi-GPU runs"}


def cfg_masked(a):
    """Masked ensemble (reference dict_ratio_experiment, big_sweep_experiments.py:546-580): tied
    SAEs of 8 dictionary sizes 512 * linspace(1, 5, 8) stacked to width 2560 on d = 512; the
    fused step skips every tile past a model's live size, so its time should track the sum of
    live sizes (3/5 of the stacked width) -- compared with the same 8 models unmasked."""
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.models.signatures import FunctionalMaskedTiedSAE, FunctionalTiedSAE

    dev = "cuda:0"
    torch.manual_seed(0)
    d, B = 512, a.batch
    sizes = [int(512 * x) for x in np.linspace(1, 5, 8)]
    stack = ((max(sizes) + 127) // 128) * 128
    ring = _ring(d, dev, rows=1 << 18)
    out = {"config": f"masked: {len(sizes)} tied SAEs of sizes {sizes} stacked to {stack}, d={d}, batch {B}",
           "unit": "activations/s", "dtype": "bf16", "data": "synthetic",
           "live_fraction": round(sum(sizes) / (stack * len(sizes)), 4)}
    variants = (("masked", FunctionalMaskedTiedSAE, lambda: [FunctionalMaskedTiedSAE.init(d, s, stack, 1e-3, device=dev)
                                                            for s in sizes]),
                ("unmasked", FunctionalTiedSAE, lambda: [FunctionalTiedSAE.init(d, stack, 1e-3, device=dev) for _ in sizes]))
    for name, sig, make in variants:
        if a.variant not in ("both", name):
            continue
        models = make()
        eng = FusedSAEEnsemble(models, sig, lr=1e-3, batch_size=B, device=dev)
        # both variants as the headline step runs: 8-step HIP graphs with the ring gather inside
        # (the per-step eager sample + single-step replay of round 3 added the same ~10 us to both)
        from sparse_coding__amd.engine.graph_plan import count_pattern

        eng.enable_graph().attach_source(ring.graph_source(B))
        pat = count_pattern(8, 8)
        eng.prime_source(patterns=[pat])
        groups, wgroups = max(1, a.steps // 8), max(1, a.warmup // 8)
        el = _timed(lambda: eng.step_source(8, pat), groups, wgroups, torch.cuda.synchronize)
        out[f"{name}_ms_per_step"] = round(1e3 * el / (8 * groups), 4)
        del eng
        torch.cuda.empty_cache()
    if a.variant == "both":
        out["time_ratio"] = round(out["masked_ms_per_step"] / out["unmasked_ms_per_step"], 4)
    out["value"] = round(B / out[f"{'unmasked' if a.variant == 'unmasked' else 'masked'}_ms_per_step"] * 1e3, 1)
    return out


def cfg_mlp(a):
    """Pythia-70m MLP hidden activations (``mlp`` = hook_post, d_mlp = 2048), ratio 4 (n = 8192),
    8-model L1 sweep, fused engine in one HIP graph; plus the per-GPU step of the
    ensemble-sharded layout at N = 2, 4, 8 (G/N models on N*B gathered rows) that the
    8-GPU run uses."""
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.models.signatures import FunctionalSAE

    dev = "cuda:0"
    torch.manual_seed(0)
    d, ratio, B = 2048, 4, a.batch
    n = d * ratio
    l1s = np.logspace(-4, -2, a.models)
    models = [FunctionalSAE.init(d, n, float(l), device=dev) for l in l1s]
    ring = _ring(d, dev, rows=1 << 18)
    out = {"config": f"Pythia-70m MLP hidden (hook_post) shapes d={d}, ratio {ratio} (n={n}), {a.models} models, fused, "
                     "per-GPU work of the 8-GPU ensemble-sharded run", "unit": "activations/s", "batch": B,
           "dtype": "bf16", "data": "synthetic", "per_n": []}
    for N in (1, 2, 4, 8):
        if a.models % N:
            continue
        gb = N * B
        eng = FusedSAEEnsemble(models[: a.models // N], FunctionalSAE, lr=1e-3, batch_size=gb, device=dev)
        eng.enable_graph()
        el = _timed(lambda: (ring.sample(gb, out=eng.x_static), eng.step_static()), a.steps, a.warmup,
                    torch.cuda.synchronize)
        ms = 1e3 * el / a.steps
        out["per_n"].append({"N": N, "models_per_gpu": a.models // N, "rows_per_step": gb, "ms_per_step": round(ms, 3),
                             "job_activations_per_s": round(gb / ms * 1e3, 1), "wgrad_split": eng.wsplit})
        del eng
        torch.cuda.empty_cache()
    out["value"] = out["per_n"][0]["job_activations_per_s"]
    return out


def cfg_harvest(a):
    """Activation harvest into the HBM ring (reference activation_dataset.py:326-391; notebook
    rate BASELINE row 7: 29.1 k act/s harvest + encode): random-init Pythia-70m / Pythia-410m
    in bf16, forward stopped after the hooked layer, [(b s), d] rows pushed into a DeviceRing;
    then the same with an 8-model SAE encode of every harvested batch."""
    from sparse_coding__amd.data.harvest import ActivationHarvester, build_model, get_activation_size
    from sparse_coding__amd.data.ring import DeviceRing
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.models.signatures import FunctionalSAE
    from sparse_coding__amd.ops import gemm

    dev = "cuda:0"
    out = {"config": "harvest: random-init LM forward -> hook -> HBM ring (+ 8-model encode)", "unit": "activations/s",
           "runs": []}
    for name, layer in (("pythia-70m", 2), ("pythia-410m", 12)):
        model = build_model(name, device=dev, dtype=torch.bfloat16)
        d = get_activation_size(name, "residual")
        h = ActivationHarvester(model, [layer], "residual")
        bs, seq = 64, 256
        toks = [torch.randint(0, 50000, (bs, seq), device=dev) for _ in range(4)]
        ring = DeviceRing(1 << 22, d, device=dev)
        it = [0]

        def harvest():
            acts = h.run(toks[it[0] % 4])[layer]
            it[0] += 1
            ring.push(acts)
            return acts

        el = _timed(harvest, a.steps, a.warmup, torch.cuda.synchronize)
        rows = bs * seq * a.steps
        rec = {"model": name, "layer": layer, "d": d, "batch_tokens": bs * seq, "harvest_act_per_s": round(rows / el, 1)}
        if d % 256 == 0:
            models = [FunctionalSAE.init(d, 4 * d, 1e-3, device=dev) for _ in range(8)]
            eng = FusedSAEEnsemble(models, FunctionalSAE, batch_size=bs * seq, device=dev)

            def harvest_encode():
                acts = harvest()
                gemm.encode_relu(acts, eng.enc_shadow, eng.params["encoder_bias"], eng.c, eng.enc_part, None, None)

            el2 = _timed(harvest_encode, a.steps, a.warmup, torch.cuda.synchronize)
            rec["harvest_plus_8model_encode_act_per_s"] = round(rows / el2, 1)
            del eng
        out["runs"].append(rec)
        h.close()
        del model, ring
        torch.cuda.empty_cache()
    out["value"] = out["runs"][0]["harvest_act_per_s"]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("which", choices=["cpu", "topk", "fista", "config5", "fistaloss", "mlp", "mlpout", "masked",
                                      "harvest"])
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--models", type=int, default=8)
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--ratio", type=float, default=1.0)
    ap.add_argument("--sparse-k", default="auto", help="topk: models with k <= this take the slot-list wgrad")
    ap.add_argument("--eager", action="store_true", help="topk: no HIP graph")
    ap.add_argument("--graph-steps", type=int, default=8,
                    help="topk: steps per graph replay with the batch gather in the graph (1: host sampling)")
    ap.add_argument("--variant", default="both", choices=["both", "masked", "unmasked"], help="masked: which run")
    ap.add_argument("--ring-gb", type=float, default=0.0,
                    help="fista: ring size in GB of HBM (0: 512k rows); config5: 0 = free memory - reserve")
    ap.add_argument("--reserve-gb", type=float, default=24.0, help="config5: HBM left outside the ring")
    a = ap.parse_args()
    rec = {"cpu": cfg_cpu, "topk": cfg_topk, "fista": cfg_fista, "config5": cfg_config5, "fistaloss": cfg_fistaloss, "mlp": cfg_mlp, "mlpout": cfg_mlpout, "masked": cfg_masked,
           "harvest": cfg_harvest}[a.which](a)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
