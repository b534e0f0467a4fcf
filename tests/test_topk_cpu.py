"""Host-side checks of the top-k front-ends (no GPU): argument validation of ``topk_select``'s score
layouts and the engine's split of models into gather-decoded and GEMM-decoded ones."""

import pytest
import torch


def test_topk_select_rejects_bad_layouts():
    from sparse_coding__amd.ops import topk as T

    k = torch.tensor([4, 8], dtype=torch.int32)
    with pytest.raises(ValueError, match="layout"):
        T.topk_select(torch.zeros(2, 16, 64, dtype=torch.bfloat16), k, 8, layout="gnb")
    with pytest.raises(ValueError, match="bf16"):
        T.topk_select(torch.zeros(16, 2, 64), k, 8, layout="bgn")  # [B, G, n] is a bf16-only layout
    with pytest.raises(ValueError, match="k must be int32"):
        T.topk_select(torch.zeros(16, 3, 64, dtype=torch.bfloat16), k, 8, layout="bgn")  # G = 3 != 2


@pytest.mark.parametrize("ks,sparse_g,gemm_k,want", [
    ([8, 16, 24, 32, 48, 64, 96, 128], 3, 0, 8),    # off
    ([8, 16, 24, 32, 48, 64, 96, 128], 3, 96, 6),   # the trailing k >= 96 models
    ([8, 16, 24, 32, 48, 64, 96, 128], 3, 8, 3),    # never below the slot-list models
    ([4, 16, 64], 0, 16, 1),
    ([64, 16, 128], 0, 32, 2),                      # a trailing RUN only (16 breaks it)
])
def test_gemm_decode_start(ks, sparse_g, gemm_k, want):
    from sparse_coding__amd.engine.topk import gemm_decode_start

    assert gemm_decode_start(ks, sparse_g, gemm_k) == want


def test_decode_grad_gemm_models_need_the_code_buffer():
    from sparse_coding__amd.ops import topk as T

    G, B, kmax, n, d = 2, 4, 8, 64, 256
    idx = torch.zeros(G, B, kmax, dtype=torch.int32)
    with pytest.raises(ValueError, match="codebuf"):
        T.decode_grad(idx, torch.zeros(G, B, kmax), torch.tensor([4, 8], dtype=torch.int32),
                      torch.zeros(G, n, d, dtype=torch.bfloat16), torch.zeros(B, d, dtype=torch.bfloat16),
                      torch.zeros(G, B, d, dtype=torch.bfloat16), torch.zeros(G, B), gemm_from=1)
