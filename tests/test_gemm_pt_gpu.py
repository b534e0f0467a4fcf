"""The persistent 128x128 tile loop (cfg bit 4: continuous LDS-DMA stream across tiles,
sae_gemm_pt_kernel) must produce bit-identical outputs to the tile kernel (cfg 1) for
every epilogue it serves, with several tiles per workgroup and with fewer tiles than
workgroup slots."""

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"
PT2, PT3 = 1 | 16, 1 | 4 | 16  # persistent, BK64 x 2 / x 3 ring


def _bf(*shape, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(torch.bfloat16)


def _step_outputs(cfg, G, B, d, n, seed):
    from sparse_coding__amd.ops import gemm

    torch.manual_seed(seed)
    x = _bf(B, d)
    we = _bf(G, n, d, scale=0.05)
    wd = torch.nn.functional.normalize(torch.randn(G, n, d, device=DEV), dim=-1).to(torch.bfloat16)
    bias = torch.randn(G, n, device=DEV) * 0.05 - 0.02
    l1 = torch.logspace(-4, -2, G, device=DEV)
    o = {}
    with gemm.force_shape(cfg):
        o["c"] = torch.empty(G, B, n, device=DEV, dtype=torch.bfloat16)
        o["part"] = torch.zeros(G, (B // 128) * (n // 128), 2, device=DEV)
        o["cnt"] = torch.zeros(G, B // 128, n, device=DEV)
        o["cmask"] = torch.zeros(gemm.code_mask_shape(G, B, n), device=DEV, dtype=torch.int64)
        gemm.encode_relu(x, we, bias, o["c"], o["part"], o["cnt"], None, mask_out=o["cmask"])
        o["r"] = torch.empty(G, B, d, device=DEV, dtype=torch.bfloat16)
        o["dpart"] = torch.zeros(G, (B // 128) * (d // 128), device=DEV)
        gemm.decode_residual(o["c"], wd, x, o["r"], o["dpart"])
        o["dpre"] = torch.empty(G, B, n, device=DEV, dtype=torch.bfloat16)
        o["colpart"] = torch.zeros(G, B // 128, n, device=DEV)
        gemm.code_grad(o["r"], wd, o["c"], l1, o["dpre"], o["colpart"], mask=o["cmask"])
        o["gd"] = torch.empty(G, n, d, device=DEV)
        o["ge"] = torch.empty(G, n, d, device=DEV)
        gemm.weight_grads([[(o["c"], o["r"])], [(o["dpre"], x)]], [o["gd"], o["ge"]], 1e-3)
        o["gt"] = torch.empty(G, n, d, device=DEV)  # tied: two K segments (K-concat)
        gemm.weight_grads([[(o["c"], o["r"]), (o["dpre"], x)]], [o["gt"]], 1e-3)
        o["nt"] = torch.empty(G, B, n, device=DEV, dtype=torch.bfloat16)
        gemm.matmul_nt(x, we, o["nt"])
    torch.cuda.synchronize()
    return o


@pytest.mark.parametrize("pcfg", [PT2, PT3])
@pytest.mark.parametrize("G,B,d,n", [(8, 2048, 512, 2048), (2, 256, 256, 512), (3, 384, 512, 640)])
def test_persistent_bit_identical(G, B, d, n, pcfg):
    ref = _step_outputs(1, G, B, d, n, seed=5)
    got = _step_outputs(pcfg, G, B, d, n, seed=5)
    for k in ref:
        assert torch.equal(got[k], ref[k]), k
