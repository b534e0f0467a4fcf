"""The kernel library's step primitives as registered PyTorch custom operators.

``ops/gemm.py`` and friends drive the gfx950 kernels through ctypes with caller-owned output
buffers (what the training engines use: nothing allocates inside a step).  This module exposes
the same kernels as functional ``torch.library`` operators in the ``sparse_coding_amd``
namespace -- typed schemas, an implementation for GPU tensors, and a fake (meta) kernel each --
so they compose with the dispatcher: shape propagation under ``FakeTensorMode`` / the meta
device, ``torch.library.opcheck``, and graph capture by tracing frontends.

    import sparse_coding__amd.ops.torch_ops  # registers the operators
    c, part, mask = torch.ops.sparse_coding_amd.sae_encode(x, w_enc, bias)

Operators (G models, B rows, d input width, n dictionary size; bf16 operands, fp32 outputs
where the engines accumulate):

* ``sae_encode(x, w, bias) -> (c, part, mask)``: c = relu(x w^T + b) bf16 [G, B, n], L1/L0
  partials, activity bitmask (``encode_relu``; reference autoencoders/sae_ensemble.py:53-56)
* ``sae_decode(c, w_hat, x) -> (r, part)``: R = c w_hat - x bf16 [G, B, d], sum R^2 partials
* ``sae_code_grad(r, w_hat, c, mask, l1) -> (dpre, colpart)``: 1[c > 0] (R w_hat^T + l1 d / 2)
* ``weight_grad(a, b, alpha) -> g``: alpha a^T b, fp32 [G, n, d] (reduction over rows)
* ``matmul_nt(a, b, alpha) -> out``: alpha a b^T, fp32 [G, M, N]
* ``rowmax_nt(a, b, alpha) -> out``: max_j alpha <a_i, b_j>, fp32 [G, M] (MMCS)
* ``topk_select(scores, k, kmax) -> (idx, val)``: exact per-row top-k with per-model k
"""

from __future__ import annotations

from typing import Tuple

import torch
from torch import Tensor

from . import gemm
from . import topk as topk_ops

NS = "sparse_coding_amd"
_bf = torch.bfloat16


def _enc_part_shape(G, B, n):
    return (G, (B // 128) * (n // 128), 2)


# ------------------------------------------------------------------ sae_encode
@torch.library.custom_op(f"{NS}::sae_encode", mutates_args=(), device_types="cuda")
def sae_encode(x: Tensor, w: Tensor, bias: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    G, n, d = w.shape
    B = x.shape[-2]
    c = torch.empty(G, B, n, device=x.device, dtype=_bf)
    part = torch.zeros(_enc_part_shape(G, B, n), device=x.device)
    mask = torch.empty(gemm.code_mask_shape(G, B, n), device=x.device, dtype=torch.int64)
    gemm.encode_relu(x.contiguous(), w.contiguous(), bias.contiguous(), c, part, mask_out=mask)
    return c, part, mask


@sae_encode.register_fake
def _sae_encode_fake(x, w, bias):
    G, n, d = w.shape
    B = x.shape[-2]
    torch._check(x.shape[-1] == d and bias.shape == (G, n))
    return (x.new_empty((G, B, n), dtype=_bf), x.new_empty(_enc_part_shape(G, B, n), dtype=torch.float32),
            x.new_empty(gemm.code_mask_shape(G, B, n), dtype=torch.int64))


# ------------------------------------------------------------------ sae_decode
@torch.library.custom_op(f"{NS}::sae_decode", mutates_args=(), device_types="cuda")
def sae_decode(c: Tensor, w_hat: Tensor, x: Tensor) -> Tuple[Tensor, Tensor]:
    G, B, n = c.shape
    d = w_hat.shape[2]
    r = torch.empty(G, B, d, device=c.device, dtype=_bf)
    part = torch.zeros(G, (B // 128) * (d // 128), device=c.device)
    gemm.decode_residual(c.contiguous(), w_hat.contiguous(), x.contiguous(), r, part)
    return r, part


@sae_decode.register_fake
def _sae_decode_fake(c, w_hat, x):
    G, B, n = c.shape
    d = w_hat.shape[2]
    torch._check(w_hat.shape[1] == n and x.shape[-1] == d)
    return c.new_empty((G, B, d), dtype=_bf), c.new_empty((G, (B // 128) * (d // 128)), dtype=torch.float32)


# ------------------------------------------------------------------ sae_code_grad
@torch.library.custom_op(f"{NS}::sae_code_grad", mutates_args=(), device_types="cuda")
def sae_code_grad(r: Tensor, w_hat: Tensor, c: Tensor, mask: Tensor, l1: Tensor) -> Tuple[Tensor, Tensor]:
    G, B, d = r.shape
    n = w_hat.shape[1]
    dpre = torch.empty(G, B, n, device=r.device, dtype=_bf)
    colpart = torch.zeros(G, B // 128, n, device=r.device)
    gemm.code_grad(r.contiguous(), w_hat.contiguous(), c.contiguous(), l1.contiguous(), dpre, colpart,
                   mask=mask.contiguous())
    return dpre, colpart


@sae_code_grad.register_fake
def _sae_code_grad_fake(r, w_hat, c, mask, l1):
    G, B, d = r.shape
    n = w_hat.shape[1]
    torch._check(c.shape == (G, B, n) and l1.shape[0] == G)
    return r.new_empty((G, B, n), dtype=_bf), r.new_empty((G, B // 128, n), dtype=torch.float32)


# ------------------------------------------------------------------ weight_grad
@torch.library.custom_op(f"{NS}::weight_grad", mutates_args=(), device_types="cuda")
def weight_grad(a: Tensor, b: Tensor, alpha: float) -> Tensor:
    G, K, n = a.shape
    d = b.shape[-1]
    out = torch.empty(G, n, d, device=a.device, dtype=torch.float32)
    gemm.weight_grads([[(a.contiguous(), b.contiguous())]], [out], float(alpha))
    return out


@weight_grad.register_fake
def _weight_grad_fake(a, b, alpha):
    G, K, n = a.shape
    torch._check(b.shape[-2] == K)
    return a.new_empty((G, n, b.shape[-1]), dtype=torch.float32)


# ------------------------------------------------------------------ matmul_nt / rowmax_nt
@torch.library.custom_op(f"{NS}::matmul_nt", mutates_args=(), device_types="cuda")
def matmul_nt(a: Tensor, b: Tensor, alpha: float) -> Tensor:
    G, N, K = b.shape
    out = torch.empty(G, a.shape[-2], N, device=a.device, dtype=torch.float32)
    gemm.matmul_nt(a.contiguous(), b.contiguous(), out, alpha=float(alpha))
    return out


@matmul_nt.register_fake
def _matmul_nt_fake(a, b, alpha):
    G, N, K = b.shape
    torch._check(a.shape[-1] == K)
    return a.new_empty((G, a.shape[-2], N), dtype=torch.float32)


@torch.library.custom_op(f"{NS}::rowmax_nt", mutates_args=(), device_types="cuda")
def rowmax_nt(a: Tensor, b: Tensor, alpha: float) -> Tensor:
    return gemm.rowmax_nt(a.contiguous(), b.contiguous(), alpha=float(alpha)).contiguous()


@rowmax_nt.register_fake
def _rowmax_nt_fake(a, b, alpha):
    torch._check(a.shape[-1] == b.shape[-1])
    return a.new_empty(a.shape[:-1], dtype=torch.float32)


# ------------------------------------------------------------------ topk_select
@torch.library.custom_op(f"{NS}::topk_select", mutates_args=(), device_types="cuda")
def topk_select(scores: Tensor, k: Tensor, kmax: int) -> Tuple[Tensor, Tensor]:
    return topk_ops.topk_select(scores.contiguous(), k.contiguous(), int(kmax))


@topk_select.register_fake
def _topk_select_fake(scores, k, kmax):
    G, B, n = scores.shape
    torch._check(k.shape[0] == G)
    return scores.new_empty((G, B, kmax), dtype=torch.int32), scores.new_empty((G, B, kmax), dtype=torch.float32)


OPS = ("sae_encode", "sae_decode", "sae_code_grad", "weight_grad", "matmul_nt", "rowmax_nt", "topk_select")
