"""CPU tests of model-level evaluation: HookedLM hook points, reconstruction
interventions, perplexity under reconstruction, ablation graphs, probe AUROC.

Parity with TransformerLens is unpinned (TransformerLens is not installed); these
pin the invariants the reference relies on: an identity reconstruction leaves the
loss unchanged, a zero intervention matches a manual splice, ablation-graph edges
follow the reference's norm/mean conventions.
"""

import os

import numpy as np

import pytest
import torch

from sparse_coding__amd.eval import interventions as I
from sparse_coding__amd.interp.hooked import HookedLM, lm_loss, parse_name, tensor_name
from sparse_coding__amd.models.learned_dict import UntiedSAE


def _tiny(arch):
    import transformers

    torch.manual_seed(0)
    if arch == "neox":
        cfg = transformers.GPTNeoXConfig(hidden_size=32, num_hidden_layers=2, num_attention_heads=4,
                                         intermediate_size=64, vocab_size=100, max_position_embeddings=64)
        return HookedLM(transformers.GPTNeoXForCausalLM(cfg).eval())
    cfg = transformers.GPT2Config(n_embd=32, n_layer=2, n_head=4, vocab_size=100, n_positions=64,
                                  bos_token_id=0, eos_token_id=0)
    return HookedLM(transformers.GPT2LMHeadModel(cfg).eval())


class _Id:
    def predict(self, x):
        return x


@pytest.mark.parametrize("arch", ["neox", "gpt2"])
def test_hook_points_and_identity_intervention(arch):
    lm = _tiny(arch)
    toks = torch.randint(0, 100, (3, 10))
    logits, cache = lm.run_with_cache(toks)
    assert cache["blocks.1.hook_resid_post"].shape == (3, 10, 32)
    assert cache["blocks.0.attn.hook_z"].shape == (3, 10, 32)
    base = lm(toks, return_type="loss")
    torch.testing.assert_close(base, lm_loss(logits, toks))
    for loc in ("residual", "mlp"):
        torch.testing.assert_close(I.perplexity_under_reconstruction(lm, _Id(), (0, loc), toks), base)
    assert parse_name(tensor_name(1, "mlp")) == (1, "mlp")


def test_residual_splice_matches_manual():
    lm = _tiny("neox")
    toks = torch.randint(0, 100, (2, 8))
    _, cache = lm.run_with_cache(toks, names_filter="blocks.1.hook_resid_post")
    final = cache["blocks.1.hook_resid_post"]

    class Half:
        def predict(self, x):
            return 0.5 * x

    got = I.run_with_model_intervention(lm, Half(), "blocks.1.hook_resid_post", toks)
    m = lm.model.gpt_neox
    want = lm.model.get_output_embeddings()(m.final_layer_norm(0.5 * final))
    torch.testing.assert_close(got, want, atol=1e-5, rtol=1e-5)


def test_ablation_graphs():
    lm = _tiny("neox")
    toks = torch.randint(0, 100, (2, 6))
    torch.manual_seed(1)
    sae = UntiedSAE(torch.randn(8, 32), torch.randn(8, 32), torch.zeros(8))
    g = I.build_ablation_graph_non_positional(lm, {(0, "residual"): sae, (1, "residual"): sae}, toks)
    assert len(g) == 16 * 16 - 16
    # manual edge: ablate feature 2 at layer 0, effect on feature 5 at layer 1
    base = I.cache_all_activations(lm, {(1, "residual"): sae}, toks)[(1, "residual")]
    abl = I.cache_all_activations(lm, {(1, "residual"): sae}, toks, fwd_hooks=[(
        "blocks.0.hook_resid_post", I.ablate_feature_intervention_non_positional(sae, (0, "residual"), 2))])[(1, "residual")]
    want = torch.norm(base[:, :, 5] - abl[:, :, 5], dim=-1).mean().item()
    assert abs(g[((0, "residual"), 2), ((1, "residual"), 5)] - want) < 1e-5
    gp = I.build_ablation_graph(lm, {(0, "residual"): sae, (1, "residual"): sae}, toks,
                                features_to_ablate={(0, "residual"): [(1, 3)]},
                                target_features={(1, "residual"): [(4, 0), (1, 3)]})
    assert len(gp) == 2 and gp[((0, "residual"), (1, 3)), ((1, "residual"), (4, 0))] >= 0


def test_calculate_perplexity_and_auroc():
    lm = _tiny("gpt2")
    batches = [torch.randint(0, 100, (2, 8)) for _ in range(2)]
    sae = UntiedSAE(torch.randn(16, 32), torch.randn(16, 32), torch.zeros(16))
    orig, recon = I.calculate_perplexity(lm, [(sae, {"l1_alpha": 1e-3})], 0, "residual", batches)
    assert orig > 1 and len(recon) == 1 and recon[0] > 1
    x = torch.randn(200, 4)
    y = (x[:, 0] > 0).long()
    assert I.logistic_regression_auroc(x, y) > 0.95


def test_scores_and_plots(tmp_path):
    import numpy as np

    from sparse_coding__amd.eval import plotting as P
    from sparse_coding__amd.eval import scores as S
    from sparse_coding__amd.models.learned_dict import TiedSAE
    from sparse_coding__amd.utils.checkpoint import save_learned_dicts

    torch.manual_seed(0)
    x = torch.randn(2000, 16)
    torch.save(x.half(), tmp_path / "0.pt")
    dicts = [(UntiedSAE(torch.randn(32, 16), torch.randn(32, 16), torch.zeros(32) - b), {"l1_alpha": a, "dict_size": 32})
             for a, b in ((1e-4, 0.0), (1e-3, 0.5), (1e-2, 1.0))]
    dicts.append((TiedSAE(torch.randn(64, 16), torch.zeros(64)), {"l1_alpha": 1e-3, "dict_size": 64}))
    save_learned_dicts(dicts, str(tmp_path / "ld.pt"))
    sample = S.load_sample(str(tmp_path / "0.pt"), n=1000)
    assert sample.shape == (1000, 16) and sample.dtype == torch.float32
    sc = S.generate_scores([("SAE", str(tmp_path / "ld.pt"))], sample, label_format="{name} {val}")
    assert list(sc) == ["SAE 32", "SAE 64"] and len(sc["SAE 32"]) == 3
    # larger negative bias -> fewer active features
    l0s = [p[0] for p in sc["SAE 32"]]
    assert l0s[0] > l0s[1] > l0s[2]
    areas = dict(S.area_under_fvu_sparsity_curve([("SAE", str(tmp_path / "ld.pt"))], sample))
    assert set(areas) == {32, 64} and all(a >= 0 for a in areas.values())
    assert len(S.scores_derivative(sc)["SAE 32"]) == 2
    rows = S.n_active_table(dicts, sample, threshold=0, with_kurtosis=True)
    assert rows[0]["frac_active"] >= rows[2]["frac_active"]
    P.plot_scores(sc, None, "L0", "FVU", (0, 40), (0, 2), "t", str(tmp_path / "g" / "fvu"))
    assert (tmp_path / "g" / "fvu.png").exists()
    P.plot_mat(np.random.rand(3, 2), [1e-3, 1e-2, 1e-1], [1, 2], save_folder=str(tmp_path), save_name="m.png")
    img = P.plot_hist(torch.randn(100), "x", "y", bins=10)
    assert img.size[0] > 0
    P.plot_capacities(dicts[:3], save_name=str(tmp_path / "cap"))
    P.plot_n_active({4: [(1e-3, 0.9), (1e-2, 0.5)]}, str(tmp_path / "na.png"))
    P.plot_violins({"a": [1.0, 2.0, 3.0], "b": []}, str(tmp_path / "v.png"))
    assert P.main(["fvu", "--dataset", str(tmp_path / "0.pt"), "--files", f"SAE={tmp_path / 'ld.pt'}",
                   "--out", str(tmp_path / "cli"), "--n", "500", "--device", "cpu"]) == 0
    assert (tmp_path / "cli.png").exists()


def test_autointerp_offline_pipeline(tmp_path):
    from sparse_coding__amd.interp.activations import (FeatureActivationDataset, make_feature_activation_dataset,
                                                       random_fragments)
    from sparse_coding__amd.interp.autointerp import (TokenListSimulator, TokenStatsExplainer, correlation_score,
                                                      interpret, parse_folder_name, read_scores)

    lm = _tiny("neox")
    torch.manual_seed(0)
    docs = [torch.randint(0, 100, (40,)) for _ in range(64)]
    frags = random_fragments(iter(docs), 60, fragment_len=16)
    assert frags.shape == (60, 16)
    sae = UntiedSAE(torch.randn(12, 32), torch.randn(12, 32), torch.zeros(12))
    ds = make_feature_activation_dataset(lm, sae, 1, "residual", frags, max_features=8, batch_size=25)
    assert ds.acts.shape == (60, 16, 8) and ds.maxes.shape == (60, 8)
    # dataset matches a direct encode
    _, cache = lm.run_with_cache(frags[:2], names_filter="blocks.1.hook_resid_post")
    want = sae.encode(cache["blocks.1.hook_resid_post"].reshape(32, 32))[:, :8].reshape(2, 16, 8)
    torch.testing.assert_close(ds.acts[:2].float(), want, atol=2e-2, rtol=1e-2)
    ds.save(str(tmp_path / "ds.pt"))
    ds2 = FeatureActivationDataset.load(str(tmp_path / "ds.pt"))
    assert torch.equal(ds2.acts, ds.acts)
    df = ds.to_dataframe()
    assert float(df["feature_3_activation_5"][7]) == float(ds.acts[7, 5, 3])
    res = interpret(ds, str(tmp_path / "res" / "sparse_coding"), 4, TokenStatsExplainer(), TokenListSimulator())
    assert len(res) >= 1 and all(-1.0 <= r["score"] <= 1.0 for r in res.values())
    scores = read_scores(str(tmp_path / "res"), "top_random")
    assert "sparse_coding" in scores and len(scores["sparse_coding"][0]) == len(res)
    assert correlation_score([[0, 1, 2]], [[0, 2, 4]]) == pytest.approx(1.0)
    assert parse_folder_name("tied_residual_l5_r0_x") == ("tied", "residual", 5, 0.5, "x")


def test_analysis_helpers():
    import numpy as np

    from sparse_coding__amd.baselines.pca import BatchedPCA
    from sparse_coding__amd.eval import analysis as A

    torch.manual_seed(0)
    lm = _tiny("gpt2")
    # a dictionary made of the token embeddings is maximally similar to them
    emb = lm.model.get_input_embeddings().weight.detach()[:20]
    d = UntiedSAE(emb.clone(), emb.clone(), torch.zeros(20))
    e, u = A.embed_unembed_similarity(lm, d)
    assert e == pytest.approx(1.0, abs=1e-5)
    small = torch.randn(8, 16)
    large = torch.cat([small[torch.randperm(8)], torch.randn(8, 16)])
    sims = A.hungarian_max_cosine(small, large)
    np.testing.assert_allclose(sims, 1.0, atol=1e-5)
    av, above, full = A.run_mmcs_with_larger([[small, large, torch.randn(32, 16)]])
    assert av[0, 0] == pytest.approx(1.0, abs=1e-5) and above[0, 0] == 100.0 and av[0, 2] == 0
    st = A.converged_feature_stats(small, large)
    assert st["frac_converged"] == 1.0
    enn = A.effective_number_of_neurons(torch.eye(4))
    assert torch.allclose(enn, torch.ones(4))
    x = torch.randn(500, 32)
    pca = BatchedPCA(32, "cpu")
    pca.train_batch(x)
    sets = A.pca_baseline_sets(pca, 32, step=8)
    sets["Added Noise"] = A.added_noise_set(32, [0.0, 0.5])
    toks = torch.randint(0, 100, (4, 8))
    res = A.fvu_vs_perplexity(lm, sets, x, toks, location=(0, "residual"), batch=2)
    assert len(res["PCA (dynamic)"]) == 2 and res["Added Noise"][0][0] == pytest.approx(0.0, abs=1e-6)
    sae = UntiedSAE(torch.randn(16, 32), torch.randn(16, 32), torch.zeros(16))
    corr = A.moment_score_correlations(sae, x, [0, 1, 2, 3], [0.1, 0.5, 0.2, 0.9])
    assert set(corr) == {"n_active", "mean", "var", "skew", "kurtosis", "l4_norm"}


def test_case_study_tools():
    from sparse_coding__amd.interp import case_studies as CS

    lm = _tiny("neox")
    torch.manual_seed(0)
    sae = UntiedSAE(torch.randn(12, 32), torch.randn(12, 32), torch.zeros(12))
    toks = torch.randint(0, 100, (3, 8))
    acts = CS.feature_activations(lm, sae, 1, "residual", toks, feature=2)
    assert acts.shape == (3, 8)
    flat = acts.flatten()
    top = CS.get_feature_datapoints(flat, 4, "max")
    assert float(flat[top[0]]) == float(flat.max())
    assert len(CS.get_feature_datapoints(flat, 4, "uniform")) >= 1
    assert CS.unravel(top[:1], 8)[0] == (int(top[0]) // 8, int(top[0]) % 8)
    eff = CS.ablate_tokens(lm, sae, 1, "residual", toks[0], 2, position=5, replacement=7)
    assert eff.shape == (6,)
    # steering: adding a tied feature's (unit) atom raises that feature's pre-activation by the scale
    from sparse_coding__amd.models.learned_dict import TiedSAE

    tied = TiedSAE(torch.randn(12, 32), torch.zeros(12) + 0.5, norm_encoder=True)
    name = "blocks.0.hook_resid_post"
    before = CS.feature_activations(lm, tied, 0, "residual", toks, feature=3)
    with lm.hooks([(name, CS.add_feature_direction(tied, 3, 5.0))]):
        _, cache = lm.run_with_cache(toks, names_filter=[name], return_type=None)
    after = tied.encode(cache[name].reshape(-1, 32))[:, 3].reshape(3, 8)
    assert (after >= before - 1e-4).all() and after.sum() > before.sum()
    d = CS.logit_diff_under(lm, toks, name, CS.ablate_feature_direction(sae, 3))
    assert d.shape == (3, 8, 100)
    up, down = CS.logit_lens(lm, sae, 3, k=5)
    assert len(up) == 5 and up[0][1] >= down[0][1]
    gen = CS.generate_text(lm, toks[:, :4], n_new=3)
    assert gen.shape == (3, 7)
    a, hi, lo = CS.best_context_token(lm, sae, 0, "residual", toks[0, :3], 3, vocab_size=100, batch_size=40)
    assert a.shape == (100,) and float(a[hi[0]]) == float(a.max())
    assert "#" in CS.render_activations(["a", "b"], [0.0, 1.0])
    assert CS.gini(torch.tensor([0.0, 0.0, 1.0])) > CS.gini(torch.ones(3))
    ld, hp = CS.select_dict([(sae, {"l1_alpha": 1e-3, "dict_size": 12})], l1_alpha=1e-3)
    assert hp["dict_size"] == 12


def test_sweep_plots(tmp_path):
    """Sweep-folder discovery + the sweep-grid, FVU-area, KL, bottleneck and auto-interp-trend
    plots (reference plotting/plot_sweep_results.py, fvu_sparsity_plot.py, plot_kl_div.py,
    bottleneck_plot.py, plot_autointerp_across_{chunks,size}.py)."""
    import torch

    from sparse_coding__amd.eval import sweep_plots as SP
    from sparse_coding__amd.models.learned_dict import TiedSAE
    from sparse_coding__amd.utils.checkpoint import save_learned_dicts

    torch.manual_seed(0)
    d = 16
    for name in ("tied_mlp_l0_r2", "untied_mlp_l0_r4", "tied_residual_l1_r2"):
        for chunk in (0, 3):
            os.makedirs(tmp_path / name / f"_{chunk}")
            lds = [(TiedSAE(torch.randn(int(d * float(name[-1])), d), torch.zeros(int(d * float(name[-1]))) - b),
                    {"l1_alpha": 1e-3 * (k + 1), "dict_size": int(d * float(name[-1]))})
                   for k, b in enumerate((0.0, 0.5, 1.0))]
            save_learned_dicts(lds, str(tmp_path / name / f"_{chunk}" / "learned_dicts.pt"))
    assert SP.parse_run_name("untied_mlpout_l3_r0.5")["loc"] == "mlpout"
    runs = SP.find_runs(str(tmp_path), loc="mlp")
    assert [m["ratio"] for m, _ in runs] == [2.0, 4.0] and all(m["chunk"] == 3 for m, _ in runs)
    sample = torch.randn(256, d)
    series = SP.sweep_series(runs, sample)
    assert len(series) == 2 and all(len(v) == 3 for v in series.values())
    grid = {(f"l{m['layer']}", m["loc"]): SP.sweep_series([(m, p)], sample) for m, p in SP.find_runs(str(tmp_path))}
    assert os.path.exists(SP.plot_sweep_grid(grid, str(tmp_path / "grid.png")))
    areas = SP.plot_fvu_sparsity_area(series, str(tmp_path / "area.png"), activation_width=d)
    assert all(np.isfinite(a) and a > 0.0 for a in areas.values())
    SP.plot_kl_div({"dict": [(0.1, 20.0), (0.3, 8.0)], "pca": [(0.2, 30.0), (0.5, 10.0)]}, str(tmp_path / "kl.png"))
    SP.plot_bottleneck({"pca": [([1, 2], 0.5, 0.1), ([1, 2, 3, 4], 0.3, 0.1)],
                        "learned_r4_1e-03": [([1], 0.4, 0.2), ([1, 2, 3], 0.1, 0.2)]}, str(tmp_path / "bn.png"), layer=2)
    m, ci = SP.mean_ci([0.1, 0.2, 0.3])
    assert abs(m - 0.2) < 1e-9 and ci > 0
    per_layer = [{"tied_r6.0_nc1": [0.1, 0.2], "tied_r6.0_nc4": [0.2, 0.25, 0.3]} for _ in range(3)]
    SP.plot_autointerp_trend(per_layer, ["tied_r6.0_nc1", "tied_r6.0_nc4"], ["0", "1", "2"], str(tmp_path / "ai.png"))
    for f in ("grid.png", "area.png", "kl.png", "bn.png", "ai.png"):
        assert (tmp_path / f).stat().st_size > 1000
