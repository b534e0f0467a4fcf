"""GPU tests of the training stack on MI355X: the sweep driver and FISTA CLI run the
fused gfx950 engines end to end, the harvester feeds the HBM ring, chunk I/O lands
in HBM."""

import os

import numpy as np
import pytest
import torch

from sparse_coding__amd.data.chunks import ChunkFolder, save_chunk
from sparse_coding__amd.engine.trainer import EnsembleTrainer
from sparse_coding__amd.models.signatures import FunctionalSAE, FunctionalTiedSAE
from sparse_coding__amd.models.topk import TopKEncoder
from sparse_coding__amd.utils import checkpoint as ckpt
from sparse_coding__amd.utils.config import SyntheticEnsembleArgs

pytestmark = pytest.mark.gpu


def _init(cfg):
    n = cfg.activation_width * 2
    ens = []
    for i, sig in enumerate((FunctionalSAE, FunctionalTiedSAE)):
        models = [sig.init(cfg.activation_width, n, float(l1)) for l1 in (1e-4, 1e-3, 3e-3)]
        ens.append((models, sig, {"batch_size": cfg.batch_size, "device": cfg.device, "dict_size": n}, f"e{i}"))
    return ens, ["dict_size"], ["l1_alpha"], {}


def test_sweep_fused_on_gpu(tmp_path):
    from sparse_coding__amd.train.sweep import sweep

    cfg = SyntheticEnsembleArgs(use_synthetic_dataset=True, activation_width=256, n_ground_truth_components=512,
                                chunk_size_gb=16384 * 256 * 2 / 1024 ** 3, n_chunks=2, batch_size=256,
                                dataset_folder=str(tmp_path / "d"), output_folder=str(tmp_path / "o"),
                                device="cuda:0", log_every=16)
    lds = sweep(_init, cfg)
    assert len(lds) == 6
    loaded = ckpt.load_learned_dicts(os.path.join(cfg.output_folder, "_1", "learned_dicts.pt"))
    x = torch.load(os.path.join(cfg.dataset_folder, "0.pt"), weights_only=True)[:4096].float()
    for ld, hp in loaded:
        ld.to_device("cpu")
        xh = ld.predict(x)
        fvu = ((xh - x) ** 2).sum() / ((x - x.mean(0)) ** 2).sum()
        assert torch.isfinite(fvu)
        if hp["l1_alpha"] < 2e-4:  # weakly regularised models learn in 128 steps; strong L1 may kill all features
            assert fvu < 0.9, (type(ld).__name__, hp, float(fvu))


def test_trainer_engines_selected():
    m = [FunctionalSAE.init(256, 512, 1e-3) for _ in range(2)]
    assert EnsembleTrainer(m, FunctionalSAE, batch_size=256, device="cuda:0").kind == "fused-sae"
    t = [TopKEncoder.init(256, 512, 8) for _ in range(2)]
    assert EnsembleTrainer(t, TopKEncoder, batch_size=256, device="cuda:0").kind == "fused-topk"
    odd = [FunctionalSAE.init(200, 512, 1e-3)]
    tr = EnsembleTrainer(odd, FunctionalSAE, batch_size=256, device="cuda:0")
    assert tr.kind == "analytic" and "not tiled" in tr.engine_reason


def test_fista_cli_on_gpu(tmp_path):
    from sparse_coding__amd.train.basic_l1_sweep import basic_l1_sweep

    g = torch.Generator().manual_seed(0)
    for i in range(2):
        save_chunk(torch.randn(4096, 256, generator=g), str(tmp_path / "d"), i)
    paths = basic_l1_sweep(str(tmp_path / "d"), str(tmp_path / "o"), 2.0, np.logspace(-4, -3, 2), batch_size=256,
                           device="cuda:0", save_after_every=True, fista_iters=50, progress=False, max_batches=4)
    assert len(paths) == 2
    lds = ckpt.load_learned_dicts(paths[-1])
    assert all(torch.isfinite(ld.get_learned_dict()).all() for ld, _ in lds)


def test_harvest_into_ring_gpu():
    from sparse_coding__amd.data.harvest import (ActivationHarvester, build_model, harvest_to_ring,
                                                 synthetic_token_batches)
    from sparse_coding__amd.data.ring import DeviceRing

    model = build_model("pythia-70m", device="cuda:0", seed=0)
    h = ActivationHarvester(model, [2], "residual")
    ring = DeviceRing(8192, 512, device="cuda:0")
    harvest_to_ring(h, synthetic_token_batches(50304, batch=8, seq_len=256), {2: ring}, 8192, device="cuda:0")
    h.close()
    assert ring.size == 8192 and torch.isfinite(ring.view().float()).all()
    assert ring.view().float().std() > 0


def test_chunk_to_hbm(tmp_path):
    x = torch.randn(20000, 512).half()
    save_chunk(x, str(tmp_path), 0)
    f = ChunkFolder(str(tmp_path))
    y = f.load(0, device="cuda:0")
    torch.cuda.synchronize()
    assert torch.equal(y.cpu(), x)


def test_huge_batch_fused_reinit(tmp_path):
    from sparse_coding__amd.data.ring import DeviceRing
    from sparse_coding__amd.train.huge_batch import HugeBatchArgs, train

    g = torch.Generator().manual_seed(0)
    for i in range(2):
        save_chunk(torch.randn(8192, 256, generator=g), str(tmp_path / "d"), i)
    cfg = HugeBatchArgs(dataset_folder=str(tmp_path / "d"), output_dir=str(tmp_path / "o"), batch_size=256,
                        n_features=512, reinit=True, reinit_every=1, device="cuda:0", log_every=8)
    tr, hist = train(cfg)
    assert tr.engine == "fused" and len(hist) == 2
    ring = DeviceRing(8192, 256, device="cuda:0")
    ring.push(torch.randn(8192, 256, generator=g).cuda())
    tr.reset_counts()
    with torch.no_grad():
        tr.impl.params["encoder_bias"][0, :7] = -1e4
    tr.impl.refresh_shadows()
    for _ in range(4):
        x, idx = ring.sample(256, return_index=True)
        tr.step(x, idx)
    assert int((tr.feature_counts() == 0).sum()) >= 7
    before = tr.impl.params["encoder"][0].clone()
    n_dead = tr.resample(ring)
    assert n_dead >= 7
    changed = (tr.impl.params["encoder"][0] != before).any(1)
    assert changed[:7].all()
    assert torch.equal(tr.impl.m["encoder"][0, :7], torch.zeros_like(tr.impl.m["encoder"][0, :7]))
    sd = torch.load(tmp_path / "o" / "sae_1.pt", weights_only=True)
    assert sd["encoder"].shape == (256, 512) and sd["decoder"].shape == (512, 256)


def _sig(kind):
    from sparse_coding__amd.models import signatures as S

    return {"untied": S.FunctionalSAE, "threshold": S.FunctionalThresholdingSAE,
            "tied_centered": S.FunctionalTiedCenteredSAE, "tied": S.FunctionalTiedSAE}[kind]


def _dp_gpu_worker(rank, world, port, x, init, kind, q, steps=3, grad_dtype=None, mode="dp"):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.parallel.data_parallel import ChunkedDataParallel, FusedChunk, split_models
    from sparse_coding__amd.parallel.dist import init_distributed, shutdown

    info = init_distributed("gloo", device="cuda:0")  # two ranks share the box's one GPU; gloo moves CUDA tensors
    torch.manual_seed(300 + rank)
    models = [({k: v.cuda() for k, v in p.items()}, {k: v.cuda() for k, v in b.items()}) for p, b in init]
    if rank:  # rank 0's parameters must win the initial broadcast
        models = [(dict((k, torch.randn_like(v)) for k, v in p.items()), b) for p, b in models]
    engines = [FusedSAEEnsemble(m, _sig(kind), lr=1e-3, batch_size=x.shape[0] // world, device="cuda:0")
               for m in split_models(models, 2)]
    gdt = grad_dtype or torch.float32
    graph = mode.endswith("_graph")
    xbuf = torch.empty(x.shape[0] // world, x.shape[1], device="cuda:0", dtype=torch.bfloat16)
    if mode.startswith("zero1"):
        from sparse_coding__amd.parallel.zero import ZeroFusedChunk

        chunks = [ZeroFusedChunk(e, info, gdt, graph=graph, x_static=xbuf) for e in engines]
    else:
        chunks = [FusedChunk(e, graph=graph, x_static=xbuf) for e in engines]
    dp = ChunkedDataParallel(chunks, info, gdt, cross_step=mode != "dp")
    xall = x.cuda()
    nb = xall.shape[0] // (world * engines[0].batch_size)
    for s_ in range(steps):  # walk the batches so a long run sees fresh rows
        blk = xall.chunk(nb)[s_ % nb] if nb > 1 else xall
        xbuf.copy_(blk.chunk(world)[rank])
        out = dp.step_batch(xbuf)
    dp.flush()
    for c in chunks:
        if hasattr(c, "gather_masters"):  # ZeRO-1: each rank owns a row shard of the masters
            c.gather_masters()
    torch.cuda.synchronize()
    res = {k: torch.cat([e.params[k] for e in engines]).cpu().numpy() for k in engines[0].params}
    if steps > 3:
        res["_loss"] = torch.cat([o[:, 0] for o in out] if isinstance(out, (list, tuple)) else [out[:, 0]]).cpu().numpy()
    q.put((rank, res))
    shutdown(info)


@pytest.mark.parametrize("kind", ["untied", "threshold", "tied_centered"])
def test_chunked_dp_fused_two_ranks_one_gpu(kind):
    """Two gloo ranks sharing cuda:0 run the chunk-pipelined fused DP step (every fused kind,
    including the threshold SAE's scale / centering and the learned center, whose gradient
    sources ride in the same flat all-reduce buffer); replicas stay identical and match
    single-process training on the global batch."""
    import socket

    import torch.multiprocessing as mp

    from sparse_coding__amd.engine.fused import FusedSAEEnsemble

    torch.manual_seed(0)
    d, n, B = 256, 512, 512
    sig = _sig(kind)
    init = [sig.init(d, n, l1) for l1 in (1e-4, 3e-4, 1e-3, 2e-3)]
    feats = torch.nn.functional.normalize(torch.randn(1024, d), dim=-1)
    x = (torch.relu(torch.randn(B, 1024) - 2.0) @ feats + 0.1).to(torch.bfloat16)
    ref = FusedSAEEnsemble([({k: v.cuda() for k, v in p.items()}, {k: v.cuda() for k, v in b.items()})
                            for p, b in init], sig, lr=1e-3, batch_size=B, device="cuda:0")
    for _ in range(3):
        ref.step_batch(x.cuda())
    torch.cuda.synchronize()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_gpu_worker, args=(r, 2, port, x, init, kind, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for k in res[0]:
        np.testing.assert_array_equal(res[0][k], res[1][k])
        want = ref.params[k].cpu().numpy()
        # bf16 GEMM partial sums differ between the half batches and the full batch: compare updates
        init_k = np.stack([p[k].numpy() for p, _ in init])
        du, dr = (res[0][k] - init_k).ravel(), (want - init_k).ravel()
        cos = float(du @ dr / (np.linalg.norm(du) * np.linalg.norm(dr) + 1e-30))
        assert cos > 0.99, (k, cos)


@pytest.mark.parametrize("mode,kind", [("dp_graph", "untied"), ("zero1", "untied"), ("zero1_graph", "untied"),
                                       ("zero1_graph", "tied")])
def test_dp_modes_two_ranks_one_gpu(mode, kind):
    """Graph-captured data parallel and ZeRO-1 (reduce-scatter -> row-sharded Adam -> shadow
    all-gather) on two gloo ranks sharing cuda:0: replicas identical after gathering the
    masters, updates match single-process training on the global batch."""
    import socket

    import torch.multiprocessing as mp

    from sparse_coding__amd.engine.fused import FusedSAEEnsemble

    torch.manual_seed(1)
    d, n, B = 256, 512, 512
    sig = _sig(kind)
    init = [sig.init(d, n, l1) for l1 in (1e-4, 3e-4, 1e-3, 2e-3)]
    feats = torch.nn.functional.normalize(torch.randn(1024, d), dim=-1)
    x = (torch.relu(torch.randn(B, 1024) - 2.0) @ feats + 0.1).to(torch.bfloat16)
    ref = FusedSAEEnsemble([({k: v.cuda() for k, v in p.items()}, {k: v.cuda() for k, v in b.items()})
                            for p, b in init], sig, lr=1e-3, batch_size=B, device="cuda:0")
    for _ in range(3):
        ref.step_batch(x.cuda())
    torch.cuda.synchronize()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_gpu_worker, args=(r, 2, port, x, init, kind, q, 3, None, mode))
             for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for k in res[0]:
        np.testing.assert_array_equal(res[0][k], res[1][k])
        want = ref.params[k].cpu().numpy()
        init_k = np.stack([p[k].numpy() for p, _ in init])
        du, dr = (res[0][k] - init_k).ravel(), (want - init_k).ravel()
        cos = float(du @ dr / (np.linalg.norm(du) * np.linalg.norm(dr) + 1e-30))
        assert cos > 0.99, (mode, k, cos)


def test_sweep_cli_ensemble_sharded_rccl(tmp_path):
    """basic_l1_sweep --parallel es under torch.distributed.run (one rank: the sharded path
    with real RCCL collectives -- batch all-gather, parameter gather for the checkpoint)."""
    import subprocess
    import sys

    g = torch.Generator().manual_seed(0)
    for i in range(2):
        save_chunk(torch.randn(4096, 256, generator=g), str(tmp_path / "d"), i)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", "29561", "-m", "sparse_coding__amd.train.basic_l1_sweep",
           "--dataset_dir", str(tmp_path / "d"), "--output_dir", str(tmp_path / "o"), "--ratio", "2.0",
           "--l1_value_n", "2", "--signature", "sae", "--batch_size", "256", "--parallel", "es",
           "--save_after_every", "false"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lds = ckpt.load_learned_dicts(str(tmp_path / "o" / "learned_dicts_epoch_0.pt"))
    assert len(lds) == 2 and all(torch.isfinite(ld.get_learned_dict()).all() for ld, _ in lds)


def test_masked_ensemble_fused_skips_dead_tiles():
    """Masked tied SAEs of several sizes stacked to one width (reference sae_ensemble.py:306-371,
    dict_ratio_experiment): the fused engine (which skips the MFMA work of tiles past each model's
    live size) tracks the eager masked signature, and parameters past dict_size never change."""
    from sparse_coding__amd.engine.ensemble import FunctionalEnsemble
    from sparse_coding__amd.engine.fused import FusedSAEEnsemble
    from sparse_coding__amd.engine.optim import adam
    from sparse_coding__amd.models.signatures import FunctionalMaskedTiedSAE

    torch.manual_seed(5)
    d, stack, B = 256, 640, 256
    sizes = [128, 256, 384, 640]
    models = [FunctionalMaskedTiedSAE.init(d, s, stack, 1e-3, device="cuda") for s in sizes]
    ref = FunctionalEnsemble([({k: v.clone() for k, v in p.items()}, b) for p, b in models], FunctionalMaskedTiedSAE,
                             adam, {"lr": 1e-3}, device="cuda")
    fused = FusedSAEEnsemble(models, FunctionalMaskedTiedSAE, lr=1e-3, batch_size=B, device="cuda")
    feats = torch.nn.functional.normalize(torch.randn(1024, d, device="cuda"), dim=-1)
    for _ in range(4):
        x = (torch.relu(torch.randn(B, 1024, device="cuda") - 2.0) @ feats).to(torch.bfloat16)
        loss_ref, _ = ref.step_batch(x.float())
        out = fused.step_batch(x)
        torch.cuda.synchronize()
        torch.testing.assert_close(out[:, 0], loss_ref["loss"], rtol=3e-2, atol=1e-4)
    init = torch.stack([p["encoder"] for p, _ in models])
    for g, s in enumerate(sizes):
        assert torch.equal(fused.params["encoder"][g, s:], init[g, s:]), g
        mv_f = (fused.params["encoder"][g, :s] - init[g, :s]).flatten()
        mv_r = (ref.params["encoder"][g, :s] - init[g, :s]).flatten()
        assert torch.nn.functional.cosine_similarity(mv_f, mv_r, dim=0).item() > 0.97, g


def test_chunked_dp_bf16_gradient_allreduce_converges():
    """The optional bf16 gradient all-reduce (half the RCCL bytes) trains like the fp32 one:
    two gloo ranks on cuda:0, 150 steps each way, replicas identical, final per-model losses
    within 3 % of the fp32 run's."""
    import socket

    import torch.multiprocessing as mp

    torch.manual_seed(1)
    d, n, B = 256, 512, 512
    sig = _sig("untied")
    init = [sig.init(d, n, l1) for l1 in (1e-4, 3e-4, 1e-3, 2e-3)]
    feats = torch.nn.functional.normalize(torch.randn(1024, d), dim=-1)
    x = (torch.relu(torch.randn(8 * B, 1024) - 2.0) @ feats + 0.1).to(torch.bfloat16)
    finals = {}
    for dt in (torch.float32, torch.bfloat16):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        procs = [ctx.Process(target=_dp_gpu_worker, args=(r, 2, port, x, init, "untied", q, 150, dt))
                 for r in range(2)]
        for p in procs:
            p.start()
        res = dict(q.get(timeout=300) for _ in procs)
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
        for k in res[0]:
            if k != "_loss":  # losses are each rank's own half batch
                np.testing.assert_array_equal(res[0][k], res[1][k])
        finals[str(dt)] = res[0]["_loss"]
    f32, b16 = finals["torch.float32"], finals["torch.bfloat16"]
    assert np.all(np.abs(b16 - f32) <= 0.03 * np.abs(f32)), (f32, b16)
