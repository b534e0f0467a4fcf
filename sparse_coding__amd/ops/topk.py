"""Host wrappers of the top-k kernels (``csrc/topk.hip``)."""

from __future__ import annotations

import os
from typing import Optional

import torch

from . import _lib


def topk_select(scores: torch.Tensor, k: torch.Tensor, kmax: int, absolute: bool = False, relu: bool = True,
                out=None, x: torch.Tensor = None, D: torch.Tensor = None):
    """Per-row top-k of ``scores`` [G, B, n] (fp32, or bf16) with per-model ``k`` (int32 [G]).

    Returns (idx int32 [G, B, kmax], val fp32 [G, B, kmax]); slots >= k[g] are (0, 0.0).
    ``absolute`` selects by |score| (PCA-style) and keeps the signed value; ``relu``
    clamps kept values at 0 (TopKEncoder semantics).  ``out``: optional (idx, val) to fill
    (contiguous, e.g. a model slice of larger buffers).

    bf16 scores (the scores GEMM's bf16 epilogue): the picks are the fp32 top-k of the scores the
    GEMM accumulated -- bf16 rounding is monotone, so only keys equal to the k-th largest bf16 key
    are ambiguous, and with ``x`` ([B, d] or [G, B, d] bf16) and ``D`` ([G, n, d] bf16, the GEMM's
    operands) those are ranked by their exact fp32 scores (ties to the lower column; without them,
    or beyond 64 such keys, by column).  Values are the bf16 scores.

    Limits of the exact-fp32 guarantee (bf16 scores): the bracket path resolves the ambiguous keys for
    k <= 256 with at most BR_CAP bracket candidates and TIE_CAP = 64 keys tied at the k-th bf16 key
    (csrc/topk.hip); past those limits the select falls back to bisection / radix on the bf16 keys and
    ties at the threshold are taken in column order -- a pick may then differ from the fp32 top-k at
    a near-tie (as it may between training, bf16 scores, and ``encode()``, fp32 scores)."""
    if scores.dim() != 3:
        raise ValueError("scores must be [G, B, n]")
    G, B, n = scores.shape
    bf = scores.dtype == torch.bfloat16
    if scores.dtype not in (torch.float32, torch.bfloat16) or not scores.is_contiguous():
        raise ValueError("scores must be contiguous fp32 or bf16")
    if k.dtype != torch.int32 or k.numel() != G:
        raise ValueError("k must be int32[G]")
    if out is not None:
        idx, val = out
        if (tuple(idx.shape) != (G, B, kmax) or tuple(val.shape) != (G, B, kmax) or idx.dtype != torch.int32
                or val.dtype != torch.float32 or not idx.is_contiguous() or not val.is_contiguous()):
            raise ValueError("out must be contiguous (int32, fp32) [G, B, kmax]")
    else:
        idx = torch.empty(G, B, kmax, device=scores.device, dtype=torch.int32)
        val = torch.empty(G, B, kmax, device=scores.device, dtype=torch.float32)
    if bf:
        sx = d = 0
        if x is not None:
            if D is None or D.dtype != torch.bfloat16 or tuple(D.shape[:2]) != (G, n) or not D.is_contiguous():
                raise ValueError("D must be contiguous bf16 [G, n, d] with x")
            d = D.shape[2]
            if (x.dtype != torch.bfloat16 or not x.is_contiguous() or x.shape[-1] != d
                    or tuple(x.shape[:-1]) not in ((B,), (G, B))):
                raise ValueError("x must be contiguous bf16 [B, d] or [G, B, d]")
            sx = B * d if x.dim() == 3 else 0
        rc = _lib.lib().sc_topk_select_bf16(_lib.ptr(scores), _lib.ptr(k), _lib.ptr(idx), _lib.ptr(val), G, B, n,
                                            kmax, int(absolute), int(relu), _lib.ptr(x), sx,
                                            _lib.ptr(D if x is not None else None), d, _lib.stream_handle())
        _lib.check(rc, "sc_topk_select_bf16")
        return idx, val
    rc = _lib.lib().sc_topk_select(_lib.ptr(scores), _lib.ptr(k), _lib.ptr(idx), _lib.ptr(val), G, B, n, kmax,
                                   int(absolute), int(relu), _lib.stream_handle())
    _lib.check(rc, "sc_topk_select")
    return idx, val


def decode_grad(idx, val, k, D, x, r_out, row_se, codebuf=None, dscbuf=None, dscv=None, prev_idx=None,
                dense_from: int = 0):
    """Sparse decode + residual (bf16 r_out [G, B, d]) + per-row squared error; with the dense
    buffers, also scatter codes and code gradients <R, D[idx]> (units of R) for the wgrad GEMM;
    with ``dscv`` ([G, B, kmax] fp32) also the per-slot code gradients for ``sparse_wgrad``.
    ``prev_idx``: the previous step's picks ([G, B, kmax]), zeroed in the dense buffers first
    (instead of a ``clear`` after the previous weight gradient).  ``dense_from``: models below it
    (slot-list weight gradient) get their per-slot ``dscv`` only -- nothing is scattered into (or
    cleared from) their dense buffers, which stay zero."""
    if prev_idx is not None and (prev_idx.shape != idx.shape or prev_idx.dtype != torch.int32
                                 or not prev_idx.is_contiguous()):
        raise ValueError("prev_idx must be contiguous int32 of idx's shape")
    G, B, kmax = idx.shape
    n, d = D.shape[1], D.shape[2]
    sx = 0 if x.dim() == 2 else B * d
    rc = _lib.lib().sc_topk_decode_grad(_lib.ptr(idx), _lib.ptr(val), _lib.ptr(k), _lib.ptr(D), _lib.ptr(x), sx,
                                        _lib.ptr(r_out), _lib.ptr(row_se), _lib.ptr(codebuf), _lib.ptr(dscbuf),
                                        G, B, n, d, kmax, _lib.stream_handle(), _lib.ptr(dscv), _lib.ptr(prev_idx),
                                        int(dense_from))
    _lib.check(rc, "sc_topk_decode_grad")


class SlotLists:
    """Device buffers of the feature-major slot lists for models [0, Gs) (``slot_lists``)."""

    def __init__(self, Gs: int, B: int, n: int, ks, kmax: int, device):
        total = B * sum(min(int(k), kmax) for k in ks[:Gs])
        self.Gs, self.B, self.n, self.kmax = Gs, B, n, kmax
        i32 = torch.int32
        self.cnt = torch.zeros(Gs * n, device=device, dtype=i32)
        self.offs = torch.zeros(Gs * n + 1, device=device, dtype=i32)
        self.cursor = torch.zeros(Gs * n, device=device, dtype=i32)
        self.tmp = torch.zeros(max(total, 1), device=device, dtype=i32)
        self.perm = torch.zeros(max(total, 1), device=device, dtype=i32)


def slot_lists(idx, k, lists: SlotLists):
    """Counting sort of the first Gs models' picks by (model, feature) on the device: afterwards
    ``lists.perm[offs[g n + j] : offs[g n + j + 1]]`` holds the slot ids (g B + b) kmax + s of
    every row b that picked feature j (s < k[g]), in increasing b.  No host synchronisation (graph
    capturable); replaces the torch sort / searchsorted of the previous host-built lists."""
    G, B, kmax = idx.shape
    if idx.dtype != torch.int32 or not idx.is_contiguous() or kmax != lists.kmax or B != lists.B:
        raise ValueError("slot_lists: idx must be contiguous int32 [G, B, kmax] matching the buffers")
    rc = _lib.lib().sc_topk_slot_lists(_lib.ptr(idx), _lib.ptr(k), _lib.ptr(lists.cnt), _lib.ptr(lists.offs),
                                       _lib.ptr(lists.cursor), _lib.ptr(lists.tmp), _lib.ptr(lists.perm), lists.Gs,
                                       B, lists.n, kmax, _lib.stream_handle())
    _lib.check(rc, "sc_topk_slot_lists")


def sparse_wgrad(lists: SlotLists, val, dscv, r, x, g_out, alpha):
    """Weight gradient of the first Gs = lists.Gs models from their picked slots only:
    g[g, j] = alpha * sum_{(b, s): idx[g, b, s] = j, s < k[g]} val R[g, b] + dscv x[b]
    (= codes^T R + dscores^T x of the dense path), summed in increasing b.  ``g_out`` fp32 or
    bf16 [Gs, n, d]."""
    Gs, n, d = g_out.shape
    _, B, kmax = val.shape
    sx = 0 if x.dim() == 2 else B * d
    rc = _lib.lib().sc_topk_sparse_wgrad(_lib.ptr(lists.perm), _lib.ptr(lists.offs), _lib.ptr(val), _lib.ptr(dscv),
                                         _lib.ptr(r), _lib.ptr(x), sx, _lib.ptr(g_out), Gs, B, n, d, kmax, float(alpha),
                                         int(g_out.dtype == torch.bfloat16), _lib.stream_handle())
    _lib.check(rc, "sc_topk_sparse_wgrad")


def clear(idx, a, b):
    G, B, kmax = idx.shape
    n = a.shape[-1]
    rc = _lib.lib().sc_topk_clear(_lib.ptr(idx), _lib.ptr(a), _lib.ptr(b), G * B, n, kmax, _lib.stream_handle())
    _lib.check(rc, "sc_topk_clear")


def scatter(idx, val, k, code):
    """Dense bf16 codes: code[g, b, idx] = val for the first k[g] slots of every row (the rest of
    ``code`` must already be zero -- ``clear`` restores that after use)."""
    G, B, kmax = idx.shape
    n = code.shape[-1]
    rc = _lib.lib().sc_topk_scatter(_lib.ptr(idx), _lib.ptr(val), _lib.ptr(k), _lib.ptr(code), G * B, B, n, kmax,
                                    _lib.stream_handle())
    _lib.check(rc, "sc_topk_scatter")
