"""CPU tests of the experiment utilities: toy-model replication grid, the minimal
ensemble example, the test-data harvester CLI, IOI prompts, per-layer baselines."""

import os
import subprocess
import sys

import numpy as np
import torch

from sparse_coding__amd.utils.checkpoint import load_learned_dicts
from sparse_coding__amd.utils.config import ToyArgs


def _toy_cfg(**kw):
    cfg = ToyArgs(activation_dim=16, n_ground_truth_components=32, batch_size=256, feature_num_nonzero=3,
                  epochs=300, device="cpu", lr=3e-3)
    return cfg.update(kw)


def test_toy_grid_ensemble_and_module_agree_on_trends():
    from sparse_coding__amd.train.toy import run_toy_grid

    l1, ratios = [1e-2, 10.0], [1, 2]
    mm, dead, rec, dicts = run_toy_grid(_toy_cfg(), l1, ratios, engine="ensemble")
    assert mm.shape == (2, 2) and dicts[1][1].shape == (64, 16)
    assert (mm > 0).all() and (mm <= 1.0 + 1e-5).all()
    assert rec[0, 0] < rec[1, 0]  # stronger L1 -> worse reconstruction
    mm2, dead2, rec2, _ = run_toy_grid(_toy_cfg(epochs=150), [1e-2], [1], engine="module")
    assert mm2.shape == (1, 1) and 0 < mm2[0, 0] <= 1.0 + 1e-5


def test_toy_main_writes_outputs(tmp_path):
    from sparse_coding__amd.train.toy import main

    out = main(["--activation_dim", "16", "--n_ground_truth_components", "32", "--batch_size", "128",
                "--epochs", "20", "--device", "cpu", "--l1_exp_low", "-2", "--l1_exp_high", "0",
                "--dict_ratio_exp_low", "0", "--dict_ratio_exp_high", "2", "--output_folder", str(tmp_path)])
    res = np.load(os.path.join(out, "results.npz"))
    assert res["mmcs"].shape == (2, 2)
    for f in ("mmcs_matrix.png", "dead_neurons_matrix.png", "av_mmcs_with_larger_dicts.png", "config.yaml"):
        assert os.path.exists(os.path.join(out, f))


def test_ensemble_example_runs():
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "examples"))
    import ensemble_training_example as ex

    tr = ex.main(["--steps", "3", "--device", "cpu", "--d", "16", "--n", "32", "--batch", "32"])
    assert tr.steps == 3


def test_generate_test_data_cli(tmp_path):
    from sparse_coding__amd.data.generate_test_data import main

    toks = torch.randint(0, 50304, (8, 16))
    torch.save(toks, tmp_path / "toks.pt")
    rc = main(["--model", "pythia-70m", "--layers", "1,2", "--dataset_folder", str(tmp_path / "acts"),
               "--chunk_size_gb", str(64 * 512 * 2 / 1024 ** 3), "--device", "cpu", "--batch_size", "2",
               "--seq_len", "16", "--token_file", str(tmp_path / "toks.pt")])
    assert rc == 0
    for L in (1, 2):
        t = torch.load(tmp_path / "acts" / f"layer_{L}" / "0.pt", weights_only=True)
        assert t.shape == (64, 512) and t.dtype == torch.float16


def test_ioi_prompts():
    from sparse_coding__amd.data.prompts import WordTokenizer, generate_ioi_dataset, ioi_logit_diff

    tok = WordTokenizer()
    b = generate_ioi_dataset(tok, 3, 2, seed=0)
    assert b.clean.shape == b.corrupted.shape == (5, b.clean.shape[1])
    for i in range(5):
        assert b.clean[i, -1] == b.answer[i]            # clean ends with the indirect object
        assert b.corrupted[i, -1] == b.distractor[i]    # corrupted ends with the subject
        assert b.answer[i] != b.distractor[i]
    assert b.clean_text[0].split(". ")[1].startswith(b.clean_text[0].split(" and ")[1].split()[0])  # ABB
    logits = torch.zeros(5, b.clean.shape[1], len(tok.vocab))
    logits[torch.arange(5), -2, b.answer] = 2.0
    assert float(ioi_logit_diff(logits, b)) == 2.0
    b2 = generate_ioi_dataset(tok, 3, 2, seed=0)
    assert torch.equal(b.clean, b2.clean)


def test_layer_baselines(tmp_path):
    from sparse_coding__amd.eval.baselines_sweep import run_layer_baselines
    from sparse_coding__amd.models.learned_dict import TiedSAE
    from sparse_coding__amd.utils.checkpoint import save_learned_dicts

    torch.manual_seed(0)
    acts = (torch.randn(3000, 16) @ torch.randn(16, 16)).half()
    os.makedirs(tmp_path / "chunks" / "l0_residual")
    torch.save(acts, tmp_path / "chunks" / "l0_residual" / "0.pt")
    sae = TiedSAE(torch.randn(32, 16), torch.zeros(32) - 0.5)
    save_learned_dicts([(sae, {"l1_alpha": 1e-3})] * 8, str(tmp_path / "sae.pt"))
    paths = run_layer_baselines(0, ["residual"], str(tmp_path / "chunks"), str(tmp_path / "out"),
                                match_dicts=str(tmp_path / "sae.pt"), match_index=7, ica_rows=1000)
    names = sorted(os.path.basename(p) for p in paths)
    assert names == ["ica.pt", "ica_topk.pt", "identity_relu.pt", "pca.pt", "pca_topk.pt", "random.pt"]
    x = acts[:100].float()
    for p in paths:
        (ld, hp), = load_learned_dicts(p)
        c = ld.encode(x)
        assert c.shape[0] == 100 and torch.isfinite(c).all(), p
    (ica, hp), = load_learned_dicts(str(tmp_path / "out" / "l0_residual" / "ica.pt"))
    assert hp["kind"] == "ica" and hp["sparsity"] > 0
    (topk, _), = load_learned_dicts(str(tmp_path / "out" / "l0_residual" / "pca_topk.pt"))
    assert int((topk.encode(x) != 0).sum(-1).max()) <= hp["sparsity"]


def test_every_run_entry_point_builds_its_sweeps(monkeypatch):
    """Every ``run_*`` runner (reference big_sweep_experiments.py:437-1286) builds configs whose
    init function returns well-formed ensembles (sweep itself stubbed out)."""
    from sparse_coding__amd.train import experiments as E
    from sparse_coding__amd.train import sweep as S

    calls = []
    monkeypatch.setattr(S, "sweep", lambda init, cfg: calls.append((init, cfg)))
    for name, fn in E.RUNS.items():
        calls.clear()
        fn(["--device", "cpu", "--activation_width", "32"])
        assert calls, name
        for init, cfg in calls[:2]:
            assert cfg.output_folder and cfg.device == "cpu", name
            ens, ens_h, buf_h, ranges = init(cfg)
            assert ens and all(len(e) == 4 and len(e[0]) >= 1 for e in ens), name
            assert isinstance(ranges, dict), name
