"""Row gather for the step's batch fetch from the HBM activation ring (``csrc/elementwise.hip``)."""

from __future__ import annotations

import torch

from . import _lib


def gather_rows(buf: torch.Tensor, idx: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """out[i] = buf[idx[i]] for a contiguous GPU ``buf`` [N, ...] whose rows are a multiple of 16 bytes;
    ``idx`` int64 on the same device.  The HIP kernel moves one row per wave."""
    if not (buf.is_cuda and buf.is_contiguous()):
        raise ValueError("gather_rows needs a contiguous GPU buffer")
    row_bytes = buf[0].numel() * buf.element_size() if buf.shape[0] else 0
    if row_bytes % 16:
        raise ValueError(f"rows of {row_bytes} bytes are not a multiple of 16")
    if idx.dtype != torch.int64 or idx.device != buf.device:
        raise ValueError("idx must be int64 on the buffer's device")
    idx = idx.contiguous()
    shape = (idx.numel(),) + tuple(buf.shape[1:])
    if out is None:
        out = torch.empty(shape, device=buf.device, dtype=buf.dtype)
    elif tuple(out.shape) != shape or out.dtype != buf.dtype or not out.is_contiguous():
        raise ValueError(f"out must be contiguous {buf.dtype} {shape}")
    rc = _lib.lib().sc_gather_rows(_lib.ptr(buf), _lib.ptr(idx), _lib.ptr(out), idx.numel(), row_bytes,
                                   _lib.stream_handle())
    _lib.check(rc, "sc_gather_rows")
    return out


def gather_rows_perm(buf: torch.Tensor, perm: torch.Tensor, step: torch.Tensor, ep0: torch.Tensor,
                     out: torch.Tensor, stride: int | None = None, offset: int = 0, inner: int | None = None,
                     ostride: int | None = None) -> torch.Tensor:
    """out[i] = buf[perm[(step - ep0) * stride + offset + i]] with ``step`` / ``ep0`` int32 [1] DEVICE
    scalars, so the fetch can be captured in a HIP graph and still walk the permutation (default
    stride = rows = out.shape[0]; data parallel: stride = N B, offset = rank B).  Several steps in one
    launch: ``inner`` rows per step, step k's rows from perm block + k ``stride`` written at output
    row k ``ostride`` (default ``inner``): out rows [k ostride, k ostride + inner).  Positions past
    ``perm`` (a host bookkeeping error) read row 0 instead of faulting."""
    if not (buf.is_cuda and buf.is_contiguous() and out.is_contiguous()):
        raise ValueError("gather_rows_perm needs contiguous GPU buffers")
    row_bytes = buf[0].numel() * buf.element_size()
    if row_bytes % 16 or tuple(out.shape[1:]) != tuple(buf.shape[1:]) or out.dtype != buf.dtype:
        raise ValueError("out rows must match buf rows (16-byte multiples)")
    if perm.dtype != torch.int64 or not perm.is_contiguous():
        raise ValueError("perm must be contiguous int64")
    for t in (step, ep0):
        if t.dtype != torch.int32 or t.numel() < 1 or t.device != buf.device:
            raise ValueError("step / ep0 must be int32 device scalars")
    inner = int(inner) if inner else None
    ostride = int(ostride) if ostride else (inner or 0)
    rows = out.shape[0] if inner is None else ((out.shape[0] - inner) // ostride + 1) * inner
    if inner is not None and ((out.shape[0] - inner) % ostride or out.shape[0] < inner):
        raise ValueError("out must hold whole strided step blocks: (k - 1) ostride + inner rows")
    stride = (out.shape[0] if inner is None else inner) if stride is None else int(stride)
    rc = _lib.lib().sc_gather_rows_perm(_lib.ptr(buf), buf.shape[0], _lib.ptr(perm), perm.numel(), _lib.ptr(step),
                                        _lib.ptr(ep0), _lib.ptr(out), rows, row_bytes, stride, int(offset),
                                        int(inner or 0), int(ostride or 0), _lib.stream_handle())
    _lib.check(rc, "sc_gather_rows_perm")
    return out


def gather_rows_blocks(buf: torch.Tensor, perm: torch.Tensor, base: int, stride: int, inner: int,
                       out: torch.Tensor) -> torch.Tensor:
    """out[o * inner + i] = buf[perm[base + o * stride + i]] for o < out.shape[0] // inner (one launch;
    e.g. rank r's shards of several consecutive data-parallel steps).  Positions past ``perm`` read
    row 0 instead of faulting."""
    if not (buf.is_cuda and buf.is_contiguous() and out.is_contiguous()):
        raise ValueError("gather_rows_blocks needs contiguous GPU buffers")
    row_bytes = buf[0].numel() * buf.element_size()
    rows = out.numel() // max(1, buf[0].numel())
    if row_bytes % 16 or out.dtype != buf.dtype or out.numel() != rows * buf[0].numel() or rows % inner:
        raise ValueError("out must hold whole rows of buf, a multiple of `inner` of them")
    if perm.dtype != torch.int64 or not perm.is_contiguous() or perm.device != buf.device:
        raise ValueError("perm must be contiguous int64 on the buffer's device")
    rc = _lib.lib().sc_gather_rows_blocks(_lib.ptr(buf), buf.shape[0], _lib.ptr(perm), perm.numel(), int(base),
                                          int(stride), int(inner), rows // inner, _lib.ptr(out), row_bytes,
                                          _lib.stream_handle())
    _lib.check(rc, "sc_gather_rows_blocks")
    return out
