"""Synthetic sparse codes on the GPU (``csrc/synth.hip``): Philox4x32-10 counter-based RNG,
per-feature Bernoulli threshold and U(0,1)*U(0,1) strengths in one elementwise kernel writing
bf16 codes, then one MFMA GEMM (``gemm.matmul_nn``) mixes them into activations -- the fused
form of reference ``sc_datasets/random_dataset.py:160-188`` (K17).  Reproducible per
(seed, row): any slice of the stream can be regenerated without the rows before it."""

from __future__ import annotations

import torch

from . import _lib


def sparse_codes(probs: torch.Tensor, batch: int, seed: int, row0: int = 0, out=None) -> torch.Tensor:
    """bf16 codes [batch, n]: code[b, j] = (u1 <= probs[j]) * u2 * u3 for stream rows
    row0 .. row0 + batch - 1."""
    n = probs.numel()
    if n % 4:
        raise ValueError("the number of features must be a multiple of 4")
    probs = probs.float().contiguous()
    if out is None:
        out = torch.empty(batch, n, device=probs.device, dtype=torch.bfloat16)
    if out.dtype != torch.bfloat16 or tuple(out.shape) != (batch, n) or not out.is_contiguous():
        raise ValueError("out must be contiguous bf16 [batch, n]")
    rc = _lib.lib().sc_synth_codes(_lib.ptr(probs), _lib.ptr(out), batch, n, int(seed) & (2**64 - 1),
                                   int(row0), _lib.stream_handle())
    _lib.check(rc, "sc_synth_codes")
    return out


def mix(codes: torch.Tensor, feats_bf16: torch.Tensor, out=None) -> torch.Tensor:
    """x = codes @ feats on the grouped MFMA GEMM (bf16 in, bf16 or fp32 out); falls back to
    torch for shapes the tile kernel does not cover."""
    from . import gemm

    B, n = codes.shape
    d = feats_bf16.shape[1]
    if out is None:
        out = torch.empty(B, d, device=codes.device, dtype=torch.bfloat16)
    if B % 128 == 0 and d % 128 == 0 and n % 64 == 0:
        gemm.matmul_nn(codes[None], feats_bf16[None].contiguous(), out[None] if out.dim() == 2 else out)
    else:
        out.copy_(codes.float() @ feats_bf16.float())
    return out
