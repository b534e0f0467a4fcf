"""Host-side checks of the top-k front-ends (no GPU): argument validation of ``topk_select``."""

import pytest
import torch


def test_topk_select_rejects_bad_shapes():
    from sparse_coding__amd.ops import topk as T

    k = torch.tensor([4, 8], dtype=torch.int32)
    with pytest.raises(ValueError, match="scores must be"):
        T.topk_select(torch.zeros(2, 16, 4, 64, dtype=torch.bfloat16), k, 8)
    with pytest.raises(ValueError, match="k must be int32"):
        T.topk_select(torch.zeros(3, 16, 64, dtype=torch.bfloat16), k, 8)  # G = 3 != 2
    with pytest.raises(ValueError, match="D must be"):
        T.topk_select(torch.zeros(2, 16, 64, dtype=torch.bfloat16), k, 8, x=torch.zeros(16, 256, dtype=torch.bfloat16))
