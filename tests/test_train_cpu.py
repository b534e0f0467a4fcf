"""CPU tests of the training stack: config, logging, chunk I/O (native reader),
harvester, trainer facade, sweep driver (+resume), experiment catalogue, the fork
CLI, and data parallelism / sweep sharding over gloo with world_size 2.

Reference test strategy: SURVEY.md section 4 (the reference has only an ad-hoc
sweep smoke test, ``test/test_sweep.py``; these pin the behaviours it relies on).
"""

import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from sparse_coding__amd.data.chunks import ChunkFolder, save_chunk, storage_extent
from sparse_coding__amd.engine.ensemble import FunctionalEnsemble
from sparse_coding__amd.engine.optim import adam
from sparse_coding__amd.engine.trainer import EnsembleTrainer
from sparse_coding__amd.models.fista import FunctionalFista
from sparse_coding__amd.models.signatures import FunctionalSAE, FunctionalTiedSAE
from sparse_coding__amd.utils import checkpoint as ckpt
from sparse_coding__amd.utils.config import (EnsembleArgs, SweepArgs, SyntheticEnsembleArgs, TrainArgs,
                                             make_hyperparam_name)
from sparse_coding__amd.utils.logging import Logger, model_metric_names


# ----------------------------------------------------------------------------- config / logging
def test_config_cli_yaml_roundtrip(tmp_path):
    cfg = EnsembleArgs.from_cli(["--tied_ae", "false", "--lr", "3e-4", "--dtype", "bfloat16", "--layer", "4"])
    assert cfg.tied_ae is False and cfg.lr == 3e-4 and cfg.dtype == torch.bfloat16 and cfg.layer == 4
    cfg2 = EnsembleArgs.from_cli(["--tied_ae", "true"])
    assert cfg2.tied_ae is True
    p = tmp_path / "c.yaml"
    cfg.to_yaml(str(p))
    back = EnsembleArgs.from_yaml(str(p))
    assert back.to_dict() == cfg.to_dict()
    # constructing never parses sys.argv (B#15) and dict(cfg) works (B#14)
    assert dict(TrainArgs())["lr"] == 1e-3
    with pytest.raises(ValueError):
        TrainArgs().update({"no_such_field": 1})
    assert make_hyperparam_name({"l1_alpha": 1e-3, "dict_size": 512}) == "l1_alpha_1.00E-03_dict_size_512"


def test_logger_jsonl(tmp_path):
    log = Logger.from_config(str(tmp_path), use_wandb=True, config={})  # wandb absent -> JSONL only
    names = model_metric_names("ens", [{"l1_alpha": 1e-3}], [{"loss": 1.5}])
    assert names == {"ens_l1_alpha_1.00E-03_loss": 1.5}
    log.log(names, 10)
    log.close()
    rec = json.loads(open(tmp_path / "metrics.jsonl").read().strip())
    assert rec["step"] == 10 and rec["ens_l1_alpha_1.00E-03_loss"] == 1.5


# ----------------------------------------------------------------------------- chunk I/O
def test_chunk_native_reader(tmp_path):
    x = torch.randn(1000, 64).half()
    save_chunk(x, str(tmp_path), 0)
    save_chunk(x[:10] * 2, str(tmp_path), 1)
    off, size = storage_extent(str(tmp_path / "0.pt"))
    assert size == x.numel() * 2 and off > 0
    f = ChunkFolder(str(tmp_path), threads=3)
    assert f.indices == [0, 1] and f.n_rows() == 1010
    h0, h1 = f.prefetch(0), f.prefetch(1)  # two reads in flight
    assert torch.equal(f.get(h1), x[:10] * 2)
    assert torch.equal(f.get(h0), x)
    # reference loader reads our chunk files
    assert torch.equal(torch.load(tmp_path / "0.pt", weights_only=True), x)


def test_chunk_saved_view_falls_back(tmp_path):
    base = torch.randn(20, 8).half()
    torch.save(base[5:10], tmp_path / "0.pt")  # a view: storage larger than the tensor
    f = ChunkFolder(str(tmp_path))
    assert torch.equal(f.load(0), base[5:10])


# ----------------------------------------------------------------------------- harvester
def test_harvester_residual_and_mlp(tmp_path):
    from sparse_coding__amd.data.harvest import (ActivationHarvester, build_model, get_activation_size,
                                                 make_tensor_name, setup_data, synthetic_token_batches)

    model = build_model("pythia-70m", device="cpu", dtype=torch.float32, seed=0)
    assert get_activation_size("pythia-70m", "mlp") == 2048
    assert make_tensor_name(2, "residual", "pythia-70m")
    h = ActivationHarvester(model, [1, 2], "mlp", out_dtype=torch.float32)
    toks = next(synthetic_token_batches(50304, batch=2, seq_len=16))
    acts = h.run(toks)
    h.close()
    assert acts[1].shape == (32, 2048) and acts[2].shape == (32, 2048)
    rows = setup_data("pythia-70m", [str(tmp_path / "a"), str(tmp_path / "b")], [0, 1], "residual", n_chunks=2,
                      device="cpu", batch_size=2, seq_len=16, rows_per_chunk=40, model=model)
    assert rows == 80
    for sub in ("a", "b"):
        f = ChunkFolder(str(tmp_path / sub))
        assert f.indices == [0, 1] and f.meta(0)[0] == (40, 512) and f.meta(0)[1] == torch.float16


# ----------------------------------------------------------------------------- trainer facade
def test_trainer_eager_matches_functional_ensemble():
    torch.manual_seed(0)
    models = [FunctionalSAE.init(32, 64, l1) for l1 in (1e-3, 1e-2)]
    ref = FunctionalEnsemble([(dict(p), dict(b)) for p, b in models], FunctionalSAE, adam, {"lr": 1e-3})
    tr = EnsembleTrainer(models, FunctionalSAE, lr=1e-3, batch_size=16, device="cpu")
    assert tr.kind == "analytic" and tr.engine_reason == "no GPU"
    x = torch.randn(16, 32)
    for _ in range(3):
        l_ref, _ = ref.step_batch(x)
        tr.step(x)
    torch.testing.assert_close(tr.last_losses["loss"], l_ref["loss"])
    lds = tr.to_learned_dicts(["dict_size"], ["l1_alpha"]) if "dict_size" in tr.args else tr.to_learned_dicts([], ["l1_alpha"])
    assert len(lds) == 2 and abs(lds[1][1]["l1_alpha"] - 1e-2) < 1e-9
    st = tr.state_dict()
    tr2 = EnsembleTrainer(models, FunctionalSAE, lr=1e-3, batch_size=16, device="cpu")
    tr2.load_state_dict(st)
    tr.step(x)
    tr2.step(x)
    torch.testing.assert_close(tr.last_losses["loss"], tr2.last_losses["loss"])


def test_trainer_fista_hook_changes_decoder():
    torch.manual_seed(0)
    models = [FunctionalFista.init(16, 32, 1e-3)]
    tr = EnsembleTrainer(models, FunctionalFista, batch_size=32, device="cpu", fista_iters=20)
    before = tr.impl.params["decoder"].detach().clone()
    tr.step(torch.randn(32, 16))
    after = tr.impl.params["decoder"].detach()
    assert not torch.allclose(before, after)
    torch.testing.assert_close(after[0].norm(dim=0), torch.ones(16), atol=1e-4, rtol=0)  # column norm (B#4)


# ----------------------------------------------------------------------------- sweep / CLI
def _tiny_init(cfg):
    n = cfg.activation_width * 2
    ens = []
    for i, sig in enumerate((FunctionalSAE, FunctionalTiedSAE)):
        models = [sig.init(cfg.activation_width, n, float(l1)) for l1 in (1e-4, 1e-3)]
        ens.append((models, sig, {"batch_size": cfg.batch_size, "device": "cpu", "dict_size": n}, f"e{i}"))
    return ens, ["dict_size"], ["l1_alpha"], {"dict_size": [n], "l1_alpha": [1e-4, 1e-3]}


def _sweep_cfg(tmp_path, **kw):
    cfg = SyntheticEnsembleArgs(use_synthetic_dataset=True, activation_width=32, n_ground_truth_components=64,
                                chunk_size_gb=64 * 32 * 2 * 8 / 1024 ** 3, n_chunks=2, gen_batch_size=128,
                                batch_size=32, dataset_folder=str(tmp_path / "data"),
                                output_folder=str(tmp_path / "out"), device="cpu", log_every=4)
    return cfg.update(kw)


def test_sweep_synthetic_end_to_end(tmp_path):
    from sparse_coding__amd.train.sweep import sweep

    cfg = _sweep_cfg(tmp_path)
    lds = sweep(_tiny_init, cfg)
    assert len(lds) == 4
    assert sorted(f for f in os.listdir(cfg.dataset_folder) if not f.startswith(".")) == ["0.pt", "1.pt"]
    # generated by us: a runner may delete it; a user's folder is refused
    from sparse_coding__amd.train.sweep import remove_synthetic_dataset

    user = tmp_path / "user_acts"
    user.mkdir()
    (user / "0.pt").write_bytes(b"not ours")
    with pytest.raises(RuntimeError, match="refusing"):
        remove_synthetic_dataset(str(user))
    assert (user / "0.pt").exists()
    last = os.path.join(cfg.output_folder, "_1", "learned_dicts.pt")
    loaded = ckpt.load_learned_dicts(last)
    np.testing.assert_allclose([hp["l1_alpha"] for _, hp in loaded], [1e-4, 1e-3, 1e-4, 1e-3], rtol=1e-6)
    assert os.path.exists(os.path.join(cfg.output_folder, "_1", "config.yaml"))
    recs = [json.loads(l) for l in open(os.path.join(cfg.output_folder, "metrics.jsonl"))]
    assert any(k.endswith("_loss") for r in recs for k in r)
    # resume: everything done -> no further training, same dictionaries
    lds2 = sweep(_tiny_init, cfg)
    assert lds2 == []


def test_sweep_resume_mid_run(tmp_path):
    from sparse_coding__amd.train import sweep as sw

    cfg = _sweep_cfg(tmp_path, n_chunks=3)
    calls = []
    orig = sw.ensemble_train_loop

    def stop_after_first(*a, **k):
        if len(calls) == 2:  # 2 ensembles per chunk: die on chunk 2
            raise KeyboardInterrupt
        calls.append(1)
        return orig(*a, **k)

    sw.ensemble_train_loop = stop_after_first
    try:
        with pytest.raises(KeyboardInterrupt):
            sw.sweep(_tiny_init, cfg)
    finally:
        sw.ensemble_train_loop = orig
    st = ckpt.load_training_state(os.path.join(cfg.output_folder, "train_state_rank0.pt"))
    assert st["extra"]["next_chunk"] == 1
    lds = sw.sweep(_tiny_init, cfg)
    assert len(lds) == 4 and os.path.exists(os.path.join(cfg.output_folder, "_2", "learned_dicts.pt"))


def test_experiment_catalogue_shapes():
    from sparse_coding__amd.train import experiments as E

    cfg = EnsembleArgs(activation_width=512, device="cpu", learned_dict_ratio=2.0)
    for name in ("tied_vs_not_experiment", "simple_setoff", "long_mlp_sweep", "thresholding_experiment",
                 "zero_l1_baseline", "run_positive_init", "fista_sweep", "pythia_1_4_b_dict"):
        ens, eh, bh, ranges = E.INIT_FUNCS[name](cfg)
        for models, sig, args, ename in ens:
            assert args["dict_size"] == models[0][0][next(iter(models[0][0]))].shape[0] or sig.__name__
            assert all(k in args for k in eh)
    ens, _, _, ranges = E.INIT_FUNCS["simple_setoff"](cfg)
    l1 = [float(m[1]["l1_alpha"]) for m in ens[0][0]]
    np.testing.assert_allclose(l1, np.concatenate([[0.0], np.logspace(-4, -2, 8)]), rtol=1e-6)
    assert E.main([]) == 2


def test_basic_l1_sweep_cli(tmp_path):
    from sparse_coding__amd.train.basic_l1_sweep import main

    for i in range(2):
        save_chunk(torch.randn(256, 16), str(tmp_path / "data"), i)
    rc = main(["--dataset_dir", str(tmp_path / "data"), "--output_dir", str(tmp_path / "o"), "--ratio", "2",
               "--l1_value_n", "2", "--batch_size", "64", "--device", "cpu", "--fista_iters", "10"])
    assert rc == 0
    files = sorted(os.listdir(tmp_path / "o"))
    assert files == ["learned_dicts_epoch_0_chunk_0.pt", "learned_dicts_epoch_0_chunk_1.pt"]
    lds = ckpt.load_learned_dicts(str(tmp_path / "o" / files[-1]))
    assert len(lds) == 2 and lds[0][0].get_learned_dict().shape == (32, 16)


# ----------------------------------------------------------------------------- gloo world_size 2
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_worker(rank, world, port, x, init, out_q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from sparse_coding__amd.parallel.data_parallel import DataParallelEnsemble
    from sparse_coding__amd.parallel.dist import init_distributed, shutdown

    info = init_distributed("gloo")
    torch.manual_seed(100 + rank)  # different init per rank: DP must broadcast rank 0's
    models = init if rank == 0 else [FunctionalSAE.init(16, 32, 1e-3) for _ in range(2)]
    ens = FunctionalEnsemble(models, FunctionalSAE, adam, {"lr": 1e-2})
    dp = DataParallelEnsemble(ens, info, bucket_bytes=1024)
    shard = x.chunk(world)[rank]
    for _ in range(3):
        dp.step_batch(shard)
    # numpy arrays pickle by value (torch tensors would go through shared memory owned by this process)
    out_q.put((rank, {k: v.detach().numpy().copy() for k, v in ens.params.items()}))
    shutdown(info)


def test_data_parallel_gloo_matches_single_process():
    torch.manual_seed(0)
    init = [FunctionalSAE.init(16, 32, 1e-3) for _ in range(2)]
    x = torch.randn(64, 16)
    single = FunctionalEnsemble([(dict(p), dict(b)) for p, b in init], FunctionalSAE, adam, {"lr": 1e-2})
    for _ in range(3):
        single.step_batch(x)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, x, init, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for k in single.params:
        np.testing.assert_array_equal(res[0][k], res[1][k])
        np.testing.assert_allclose(res[0][k], single.params[k].detach().numpy(), atol=2e-5, rtol=1e-4)


def _shard_worker(rank, world, port, tmp, out_q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from sparse_coding__amd.parallel.dist import init_distributed, shutdown
    from sparse_coding__amd.train.sweep import sweep

    info = init_distributed("gloo")
    cfg = _sweep_cfg(tmp)
    lds = sweep(_tiny_init, cfg, info)
    out_q.put((rank, [type(ld).__name__ for ld, _ in lds]))
    shutdown(info)


def test_sweep_sharded_over_two_ranks(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, 2, port, tmp_path, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == ["UntiedSAE", "UntiedSAE"] and res[1] == ["TiedSAE", "TiedSAE"]
    out = tmp_path / "out" / "_1"
    assert (out / "learned_dicts_rank0.pt").exists() and (out / "learned_dicts_rank1.pt").exists()


# ----------------------------------------------------------------------------- huge-batch DP + resampling
def test_worst_indices_and_resample():
    from sparse_coding__amd.train.huge_batch import WorstIndices, resample_dead

    w = WorstIndices(3, "cpu")
    w.update(torch.tensor([0, 1, 2, 3]), torch.tensor([0.1, 0.9, 0.5, 0.2]))
    w.update(torch.tensor([7, 8]), torch.tensor([0.7, 0.05]))
    assert w.get_worst(2).tolist() == [1, 7] and w.get_worst(5).tolist() == [1, 7, 2]
    enc = torch.ones(5, 4)
    m = torch.ones(5, 4)
    vecs = torch.arange(8.0).view(2, 4)
    n = resample_dead(enc, torch.tensor([1, 3, 4]), vecs, [m])
    assert n == 2 and torch.equal(m[1], torch.zeros(4)) and torch.equal(m[4], torch.ones(4))
    torch.testing.assert_close(enc[3], vecs[1] * 0.2 / 2.0)


def test_huge_batch_torch_engine_reinit(tmp_path):
    from sparse_coding__amd.train.huge_batch import HugeBatchArgs, train

    for i in range(2):
        save_chunk(torch.randn(512, 16), str(tmp_path / "d"), i)
    cfg = HugeBatchArgs(dataset_folder=str(tmp_path / "d"), output_dir=str(tmp_path / "o"), batch_size=64,
                        n_features=32, reinit=True, reinit_every=1, device="cpu", l1_alpha=0.5, log_every=2)
    tr, hist = train(cfg)
    assert tr.engine == "torch" and all("n_dead_feats" in h for h in hist)
    # force 5 dead features, then resample them from the worst-reconstructed rows
    from sparse_coding__amd.data.ring import DeviceRing

    ring = DeviceRing(512, 16, device="cpu", dtype=torch.float32)
    ring.push(torch.randn(512, 16))
    tr.reset_counts()
    with torch.no_grad():
        tr.module.threshold[:5] = -1e4
    for _ in range(4):
        x, idx = ring.sample(64, return_index=True)
        tr.step(x, idx)
    before = tr.module.encoder.detach().clone()
    assert tr.resample(ring) == 5
    changed = (tr.module.encoder.detach() != before).any(0)
    assert changed[:5].all() and not changed[5:].any()
    sd = torch.load(tmp_path / "o" / "sae_1.pt", weights_only=True)
    assert set(sd) == {"decoder", "encoder", "threshold", "centering"} and sd["encoder"].shape == (16, 32)


def _huge_worker(rank, world, port, folder, out, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from sparse_coding__amd.parallel.dist import init_distributed, shutdown
    from sparse_coding__amd.train.huge_batch import HugeBatchArgs, train

    info = init_distributed("gloo")
    cfg = HugeBatchArgs(dataset_folder=folder, output_dir=out, batch_size=32, n_features=32, reinit=True,
                        reinit_every=1, device="cpu", l1_alpha=0.5, log_every=0)
    tr, hist = train(cfg, info)
    q.put((rank, tr.module.encoder.detach().numpy().copy(), hist[-1]["n_dead_feats"]))
    shutdown(info)


def test_huge_batch_ddp_gloo_two_ranks(tmp_path):
    for i in range(2):
        save_chunk(torch.randn(256, 16), str(tmp_path / "d"), i)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_huge_worker, args=(r, 2, port, str(tmp_path / "d"), str(tmp_path / "o"), q))
             for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (enc, nd) for r, enc, nd in (q.get(timeout=240) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    np.testing.assert_array_equal(res[0][0], res[1][0])  # replicas identical after DDP + resampling
    assert res[0][1] == res[1][1]


def _chunked_worker(rank, world, port, x, init, out_q, cross=False):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from sparse_coding__amd.parallel.data_parallel import ChunkedDataParallel, EagerChunk, split_models
    from sparse_coding__amd.parallel.dist import init_distributed, shutdown

    info = init_distributed("gloo")
    torch.manual_seed(200 + rank)  # different params per rank (DP must broadcast rank 0's), same hyper-params
    models = init if rank == 0 else [FunctionalSAE.init(16, 32, float(b["l1_alpha"])) for _, b in init]
    chunks = [EagerChunk(FunctionalEnsemble(m, FunctionalSAE, adam, {"lr": 1e-2})) for m in split_models(models, 3)]
    dp = ChunkedDataParallel(chunks, info, cross_step=cross)
    for _ in range(3):
        dp.step_batch(x.chunk(world)[rank])
    dp.flush()
    enc = torch.cat([c.ens.params["encoder"].detach() for c in chunks]).numpy().copy()
    out_q.put((rank, enc))
    shutdown(info)


@pytest.mark.parametrize("cross", [False, True])
def test_chunked_data_parallel_gloo_matches_single_process(cross):
    torch.manual_seed(0)
    init = [FunctionalSAE.init(16, 32, l1) for l1 in (1e-4, 3e-4, 1e-3, 1e-3)]  # no dead features: Adam would amplify rounding
    x = torch.randn(64, 16)
    single = FunctionalEnsemble([(dict(p), dict(b)) for p, b in init], FunctionalSAE, adam, {"lr": 1e-2})
    for _ in range(3):
        single.step_batch(x)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_chunked_worker, args=(r, 2, port, x, init, q, cross)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    np.testing.assert_array_equal(res[0], res[1])
    np.testing.assert_allclose(res[0], single.params["encoder"].detach().numpy(), atol=2e-5, rtol=1e-4)


def _job(x, device=None, progress=None):
    progress.value += 1
    return x * 2, device


def test_launcher_and_dispatch(tmp_path):
    from sparse_coding__amd.train.launch import dispatch, launch

    script = tmp_path / "rank.py"
    script.write_text("import os, sys\nopen(sys.argv[1] + '/r' + os.environ['RANK'], 'w').write("
                      "os.environ['WORLD_SIZE'] + ' ' + os.environ['MASTER_ADDR'])\n")
    codes = launch(str(script), 3, [str(tmp_path)], module=False, timeout=60)
    assert codes == [0, 0, 0]
    assert sorted(p.name for p in tmp_path.glob("r[0-9]")) == ["r0", "r1", "r2"]
    assert (tmp_path / "r1").read_text() == "3 127.0.0.1"
    res = dispatch([(_job, (i,), {}) for i in range(5)], ["cpu:a", "cpu:b"])
    assert [r for r, _ in res] and [r[0] for r, _ in res] == [0, 2, 4, 6, 8]
    assert {r[1] for r, _ in res} <= {"cpu:a", "cpu:b"}


def test_remote_command_builders(monkeypatch):
    from sparse_coding__amd.utils import remote as R

    monkeypatch.setenv("SC_REMOTE_HOST", "user@box")
    cmd = R.rsync_push(".", remote_dir="proj", port=2222)
    assert cmd[:2] == ["rsync", "-rv"] and cmd[-1] == "user@box:proj" and "ssh -p 2222" in cmd
    assert R.scp_push(["a", "b"], remote_dir="d")[-1] == "user@box:d"
    assert R.run(["echo", "x"], dry_run=True) == 0
    d = R.dotdict(a=1)
    d.b = 2
    assert d.a == 1 and d["b"] == 2 and d.c is None
    with pytest.raises(RuntimeError):
        R.upload_to_s3(__file__, bucket="b")


def test_log_standard_metrics_images(tmp_path):
    from sparse_coding__amd.models.learned_dict import TiedSAE
    from sparse_coding__amd.train.sweep import filter_learned_dicts, log_standard_metrics

    torch.manual_seed(0)
    lds = [(TiedSAE(torch.randn(n, 8), torch.zeros(n) - 0.1, norm_encoder=True), {"l1_alpha": l1, "dict_size": n})
           for n in (16, 32) for l1 in (1e-3, 1e-2)]
    assert len(filter_learned_dicts(lds, {"dict_size": 16})) == 2
    log = log_standard_metrics(lds, torch.randn(500, 8), 0, {"l1_alpha": [1e-3, 1e-2], "dict_size": [16, 32]},
                               None, str(tmp_path / "img"))
    assert 0 < log["l1_alpha_1.00E-03_dict_size_16_prop_active"] <= 1
    files = sorted(p.name for p in (tmp_path / "img").iterdir())
    assert any(f.startswith("mmcs_grid_0") for f in files) and sum(f.startswith("sparsity_hist") for f in files) == 4


# ----------------------------------------------------------------------------- ensemble-axis sharding
def _es_worker(rank, world, port, xs, init, out_q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from sparse_coding__amd.engine.analytic import AnalyticSAEEnsemble
    from sparse_coding__amd.parallel.dist import init_distributed, shutdown
    from sparse_coding__amd.parallel.ensemble_shard import EnsembleSharded

    info = init_distributed("gloo")
    es = EnsembleSharded(init, lambda m, bs: AnalyticSAEEnsemble(m, FunctionalSAE, lr=1e-2), info,
                         batch_per_rank=xs[0].shape[0] // world, d=16, dtype=torch.float32)
    assert es.engine.n_models == len(init) // world
    es.step_batch(xs[0].chunk(world)[rank])             # synchronous gather
    it = iter(xs[1:])                                   # a stateful sampler, like the ring's
    for _ in range(2):                                  # overlapped gather of the next batch
        es.step_sampled(lambda out: out.copy_(next(it).chunk(world)[rank]))
    es.flush()
    full = es.gather_params()
    lds = es.to_learned_dicts([b for _, b in init], FunctionalSAE)
    out_q.put((rank, {k: v.numpy().copy() for k, v in full.items()}, len(lds)))
    shutdown(info)


def test_ensemble_sharded_gloo_matches_global_batch():
    """Each rank trains half the models on the all-gathered batch: identical to training
    every model on the global batch in one process."""
    from sparse_coding__amd.engine.analytic import AnalyticSAEEnsemble

    torch.manual_seed(0)
    init = [FunctionalSAE.init(16, 32, l1) for l1 in (1e-4, 3e-4, 1e-3, 3e-3)]
    xs = [torch.randn(64, 16) for _ in range(4)]
    single = AnalyticSAEEnsemble([(dict(p), dict(b)) for p, b in init], FunctionalSAE, lr=1e-2)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_es_worker, args=(r, 2, port, xs, init, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, params, n = q.get(timeout=180)
        res[r] = params
        assert n == 4
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # step_sampled steps on the previously gathered batch: the workers trained on xs[0],
    # xs[1], xs[2] (xs[3] was prefetched by the last call and is never stepped)
    for x in xs[:3]:
        single.step_batch(x)
    for k in single.params:
        np.testing.assert_array_equal(res[0][k], res[1][k])
        np.testing.assert_allclose(res[0][k], single.params[k].numpy(), atol=2e-5, rtol=1e-4)


def _ring(rows, seed=7):
    from sparse_coding__amd.data.ring import DeviceRing

    r = DeviceRing(rows.shape[0], rows.shape[1], device="cpu", dtype=torch.float32, seed=seed)
    r.push(rows)
    return r


def _es_groups_worker(rank, world, port, rows, init, groups, B, out_q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from sparse_coding__amd.engine.analytic import AnalyticSAEEnsemble
    from sparse_coding__amd.parallel.dist import init_distributed, shutdown
    from sparse_coding__amd.parallel.ensemble_shard import EnsembleSharded

    info = init_distributed("gloo")
    ring = _ring(rows)  # every rank walks the same permutation and keeps its own shard of it
    es = EnsembleSharded(init, lambda m, bs: AnalyticSAEEnsemble(m, FunctionalSAE, lr=1e-2), info,
                         batch_per_rank=B, d=rows.shape[1], dtype=torch.float32)
    for chunk in groups:  # several calls, several groups per call (the bench's warmup / timed split)
        es.run_groups(chunk, lambda out, s: ring.sample_shard_steps(B, rank, world, s, out))
    full = es.gather_params()
    out_q.put((rank, {k: v.numpy().copy() for k, v in full.items()}))
    shutdown(info)


@pytest.mark.parametrize("world", [2, 4])
def test_ensemble_sharded_multistep_groups_gloo(world):
    """Multi-step groups (one local-row gather per group, per-step batch all-gathers issued under the
    previous group, one replay per group) over 2 and 4 gloo ranks == one process training every model
    on the same global batches (the ring's data-parallel permutation, rank-ordered shards)."""
    from sparse_coding__amd.engine.analytic import AnalyticSAEEnsemble

    torch.manual_seed(3)
    d, B = 16, 8
    init = [FunctionalSAE.init(d, 32, l1) for l1 in (1e-4, 3e-4, 1e-3, 3e-3)]
    rows = torch.randn(400, d)
    groups = [[3, 2], [3], [1, 4]]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_es_groups_worker, args=(r, world, port, rows, init, groups, B, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    single = AnalyticSAEEnsemble([(dict(p), dict(b)) for p, b in init], FunctionalSAE, lr=1e-2)
    ring = _ring(rows)
    for chunk in groups:
        for s in chunk:
            xs = ring.sample_shard_steps(B * world, 0, 1, s, torch.empty(s * B * world, d))
            for x in xs.view(s, B * world, d):
                single.step_batch(x)
    for k in single.params:
        for r in range(1, world):
            np.testing.assert_array_equal(res[0][k], res[r][k])
        np.testing.assert_allclose(res[0][k], single.params[k].numpy(), atol=2e-5, rtol=1e-4)


def _trainer_es_worker(rank, world, port, xs, init, out_q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from sparse_coding__amd.parallel.dist import init_distributed, shutdown

    info = init_distributed("gloo")
    tr = EnsembleTrainer(init, FunctionalSAE, lr=1e-2, batch_size=xs[0].shape[0] // world, device="cpu",
                         dist=info, parallel="es", args={"dict_size": 32})
    assert tr.kind == "analytic" and tr.impl.n_models == len(init) // world
    for x in xs:
        tr.step(x.chunk(world)[rank])
    lds = tr.to_learned_dicts(["dict_size"], ["l1_alpha"])
    out_q.put((rank, [ld.encoder.numpy().copy() for ld, _ in lds], [hp for _, hp in lds]))
    shutdown(info)


def test_trainer_ensemble_sharded_gloo():
    """EnsembleTrainer(parallel="es") over two gloo ranks == one process training every
    model on the global batch; LearnedDicts and hyper-parameters come back for all models."""
    from sparse_coding__amd.engine.analytic import AnalyticSAEEnsemble

    torch.manual_seed(1)
    init = [FunctionalSAE.init(16, 32, l1) for l1 in (1e-4, 3e-4, 1e-3, 3e-3)]
    xs = [torch.randn(64, 16) for _ in range(3)]
    single = AnalyticSAEEnsemble([(dict(p), dict(b)) for p, b in init], FunctionalSAE, lr=1e-2)
    for x in xs:
        single.step_batch(x)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_trainer_es_worker, args=(r, 2, port, xs, init, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, encs, hps = q.get(timeout=180)
        res[r] = (encs, hps)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    encs, hps = res[0]
    assert len(encs) == 4 and [h["l1_alpha"] for h in hps] == pytest.approx([1e-4, 3e-4, 1e-3, 3e-3])
    for g in range(4):
        np.testing.assert_array_equal(encs[g], res[1][0][g])
        np.testing.assert_allclose(encs[g], single.params["encoder"][g].numpy(), atol=2e-5, rtol=1e-4)


def _trainer_dp_worker(rank, world, port, xs, init, mode, out_q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from sparse_coding__amd.parallel.dist import init_distributed, shutdown

    info = init_distributed("gloo")
    tr = EnsembleTrainer(init, FunctionalSAE, lr=1e-2, batch_size=xs[0].shape[0] // world, device="cpu",
                         dist=info, parallel=mode, args={"dict_size": 32})
    assert tr.kind == f"{mode}-eager"
    for x in xs:
        tr.step(x.chunk(world)[rank])
    lds = tr.to_learned_dicts(["dict_size"], ["l1_alpha"])
    out_q.put((rank, [ld.encoder.numpy().copy() for ld, _ in lds]))
    shutdown(info)


@pytest.mark.parametrize("mode", ["dp", "zero1"])
def test_trainer_data_parallel_gloo(mode):
    """EnsembleTrainer(parallel='dp' / 'zero1') over two gloo ranks == one process training every
    model on the global batch."""
    torch.manual_seed(4)
    init = [FunctionalSAE.init(16, 32, l1) for l1 in (1e-4, 1e-3, 3e-3)]
    xs = [torch.randn(64, 16) for _ in range(3)]
    single = EnsembleTrainer(init, FunctionalSAE, lr=1e-2, batch_size=64, device="cpu", engine="eager")
    for x in xs:
        single.step(x)
    ref = [single.impl.params["encoder"][i].detach().numpy() for i in range(3)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_trainer_dp_worker, args=(r, 2, port, xs, init, mode, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for i in range(3):
        np.testing.assert_array_equal(res[0][i], res[1][i])
        np.testing.assert_allclose(res[0][i], ref[i], atol=2e-5, rtol=1e-4)
