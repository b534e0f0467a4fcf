"""The registered ``sparse_coding_amd`` operators (ops/torch_ops.py): schemas and fake (meta)
kernels, checked without a GPU -- shape / dtype propagation on the meta device."""

import torch

from sparse_coding__amd.ops import gemm
from sparse_coding__amd.ops import torch_ops

OPS = torch.ops.sparse_coding_amd


def test_operators_registered_with_schemas():
    for name in torch_ops.OPS:
        schema = str(getattr(OPS, name).default._schema)
        assert schema.startswith(f"sparse_coding_amd::{name}("), schema
        assert "!" not in schema  # functional: no mutated arguments


def test_fake_kernels_propagate_shapes_on_meta():
    G, B, d, n, k = 3, 256, 128, 512, 16
    bf, f32 = torch.bfloat16, torch.float32
    x = torch.empty(B, d, device="meta", dtype=bf)
    w = torch.empty(G, n, d, device="meta", dtype=bf)
    bias = torch.empty(G, n, device="meta", dtype=f32)
    c, part, mask = OPS.sae_encode(x, w, bias)
    assert (c.shape, c.dtype) == ((G, B, n), bf)
    assert part.shape == (G, (B // 128) * (n // 128), 2) and mask.shape == gemm.code_mask_shape(G, B, n)
    r, dpart = OPS.sae_decode(c, w, x)
    assert (r.shape, r.dtype, dpart.shape) == ((G, B, d), bf, (G, (B // 128) * (d // 128)))
    dpre, colpart = OPS.sae_code_grad(r, w, c, mask, torch.empty(G, device="meta"))
    assert (dpre.shape, colpart.shape) == ((G, B, n), (G, B // 128, n))
    g = OPS.weight_grad(c, r, 0.5)
    assert (g.shape, g.dtype) == ((G, n, d), f32)
    s = OPS.matmul_nt(x, w, 1.0)
    assert (s.shape, s.dtype) == ((G, B, n), f32)
    assert OPS.rowmax_nt(w, w, 1.0).shape == (G, n)
    idx, val = OPS.topk_select(s, torch.empty(G, device="meta", dtype=torch.int32), k)
    assert (idx.shape, idx.dtype, val.dtype) == ((G, B, k), torch.int32, f32)
