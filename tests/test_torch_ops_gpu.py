"""The registered ``sparse_coding_amd`` operators on the GPU: ``torch.library.opcheck`` (schema,
fake-kernel agreement with the real kernel, dispatcher registration) and numerics against plain
PyTorch fp32 references of the same ops."""

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from sparse_coding__amd.ops import _lib as L

    L.lib()  # must load: no silent fallback on a GPU box
    yield


def _inputs():
    torch.manual_seed(0)
    G, B, d, n = 2, 256, 256, 512
    x = torch.randn(B, d, device=DEV).to(torch.bfloat16)
    w = torch.nn.functional.normalize(torch.randn(G, n, d, device=DEV), dim=-1).to(torch.bfloat16)
    bias = torch.randn(G, n, device=DEV) * 0.05
    return x, w, bias


def test_opcheck_and_numerics():
    from sparse_coding__amd.ops import torch_ops  # noqa: F401  (registers the operators)

    OPS = torch.ops.sparse_coding_amd
    x, w, bias = _inputs()
    G, n, d = w.shape
    l1 = torch.tensor([1e-3, 3e-3], device=DEV)
    c, part, mask = OPS.sae_encode(x, w, bias)
    r, dpart = OPS.sae_decode(c, w, x)
    dpre, colpart = OPS.sae_code_grad(r, w, c, mask, l1)
    g = OPS.weight_grad(c, r, 0.5)
    s = OPS.matmul_nt(x, w, 1.0)
    mx = OPS.rowmax_nt(w, w, 1.0)
    idx, val = OPS.topk_select(s, torch.tensor([8, 16], device=DEV, dtype=torch.int32), 16)
    torch.cuda.synchronize()
    xf, wf = x.float(), w.float()
    cref = torch.relu(xf @ wf.transpose(1, 2) + bias[:, None])
    assert float((c.float() - cref).norm() / cref.norm()) < 1e-2
    rref = c.float() @ wf - xf
    assert float((r.float() - rref).norm() / rref.norm()) < 1e-2
    dref = (r.float() @ wf.transpose(1, 2) + (l1 * d / 2)[:, None, None]) * (c.float() > 0)
    assert float((dpre.float() - dref).norm() / dref.norm()) < 1e-2
    gref = 0.5 * c.float().transpose(1, 2) @ r.float()
    torch.testing.assert_close(g, gref, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(s, xf @ wf.transpose(1, 2), rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(mx, (wf @ wf.transpose(1, 2)).amax(-1), rtol=1e-2, atol=1e-2)
    ref_top = torch.topk(s[1], 16, dim=-1).values.clamp_min(0)
    torch.testing.assert_close(val[1].sort(-1, descending=True).values, ref_top, rtol=0, atol=0)
    assert not val[0, :, 8:].any()
    for op, args in ((OPS.sae_encode, (x, w, bias)), (OPS.sae_decode, (c, w, x)),
                     (OPS.sae_code_grad, (r, w, c, mask, l1)), (OPS.weight_grad, (c, r, 0.5)),
                     (OPS.matmul_nt, (x, w, 1.0)), (OPS.rowmax_nt, (w, w, 1.0))):
        torch.library.opcheck(op.default, args, test_utils=("test_schema", "test_faketensor"))
