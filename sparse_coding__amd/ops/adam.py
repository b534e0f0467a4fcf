"""Python front-end for the fused Adam / shadow / bias-loss kernels (``csrc/adam.hip``)."""

from __future__ import annotations

import ctypes as C

import torch

from . import _lib


def _vp(seq):
    return (C.c_void_p * len(seq))(*[_lib.ptr(t) for t in seq])


def adam_rows(sets, lr, step, b1=0.9, b2=0.999, eps=1e-8, rows_per_model=None, step_dev=None, nsplit=1,
              gstride=0, row0=0, live=None):
    """Fused row-wise Adam over one or two parameter sets.

    sets: list of dicts with keys p, g, m, v (fp32 [G, n, d]; ``g`` may instead be bf16 -- then
    every set's must be), shadow (bf16 [G, n, d] or None),
    norms (fp32 [G, n] or None), norm (bool: parameter is row-normalised inside the loss).
    lr: fp32 tensor [G] (per-model learning rate); step: 1-based Adam step (host value), or
    ``step_dev``: int32 device counter of completed steps (the kernel uses ``*step_dev + 1``;
    graph-capturable).  ``nsplit`` > 1: each ``g`` is the first of ``nsplit`` split-K partial
    slabs ``gstride`` elements apart, summed in the kernel.  ``row0``: global index of the
    sets' first row (row-sharded updates; the per-model lr is ``lr[(row0 + row) // n]``).
    Tensors may be [G, n, d] or [rows, d] (then pass ``rows_per_model``).  ``live``: optional
    int32 [G] live row count per model (masked ensembles; rows past it have zero gradient and
    are skipped -- their Adam update is exactly zero).
    """
    if not 1 <= len(sets) <= 2:
        raise ValueError("1 or 2 parameter sets")
    shp = tuple(sets[0]["p"].shape)
    d = shp[-1]
    nrows = sets[0]["p"].numel() // d
    n = shp[1] if len(shp) == 3 else None
    gbf16 = sets[0]["g"].dtype == torch.bfloat16
    gsize = 2 if gbf16 else 4
    for s in sets:
        for k in ("p", "g", "m", "v"):
            t = s[k]
            want = torch.bfloat16 if (k == "g" and gbf16) else torch.float32
            if t.dtype != want or tuple(t.shape) != tuple(sets[0]["p"].shape) or not t.is_contiguous():
                raise ValueError(f"adam set tensor {k} must be contiguous {want} {shp} (bf16 gradients: all sets)")
        if s.get("shadow") is not None and (s["shadow"].dtype != torch.bfloat16 or s["shadow"].numel() != nrows * d):
            raise ValueError("shadow must be bf16 of the parameter's size")
        if s.get("norms") is not None and s["norms"].numel() != nrows:
            raise ValueError("norms must have one entry per row")
        if nsplit > 1 and s["g"].untyped_storage().nbytes() < (s["g"].storage_offset() + (nsplit - 1) * gstride
                                                               + nrows * d) * gsize:
            raise ValueError("gradient storage too small for nsplit slabs")
    rpm = rows_per_model or n
    if not rpm:
        raise ValueError("rows_per_model is required for 2-D parameter sets")
    rows = (C.c_int * len(sets))(*[nrows for _ in sets])
    norm = (C.c_int * len(sets))(*[int(bool(s["norm"])) for s in sets])
    bc1 = 1.0 - b1 ** step
    bc2 = 1.0 - b2 ** step
    rc = _lib.lib().sc_adam_rows(
        len(sets), _vp([s["p"] for s in sets]), _vp([s["g"] for s in sets]),
        _vp([s["m"] for s in sets]), _vp([s["v"] for s in sets]),
        _vp([s.get("shadow") for s in sets]), _vp([s.get("norms") for s in sets]),
        rows, norm, d, rpm, _lib.ptr(lr), b1, b2, eps, bc1, bc2,
        _lib.ptr(step_dev), int(nsplit), int(gstride), int(row0), _lib.stream_handle(), _lib.ptr(live),
        int(gbf16),
    )
    _lib.check(rc, "sc_adam_rows")


def shadow_rows(p, shadow, norms=None, normalize=True):
    """bf16 shadow (row-normalised if ``normalize``) of fp32 rows p[..., d]."""
    d = p.shape[-1]
    rows = p.numel() // d
    if not (p.is_contiguous() and shadow.is_contiguous() and shadow.dtype == torch.bfloat16):
        raise ValueError("shadow_rows needs contiguous fp32 p and bf16 shadow")
    rc = _lib.lib().sc_shadow_rows(_lib.ptr(p), _lib.ptr(shadow), _lib.ptr(norms), rows, d,
                                   int(normalize), _lib.stream_handle())
    _lib.check(rc, "sc_shadow_rows")


def bias_loss(b, m, v, colpart, tm, enc_part, enc_tiles, dec_part, dec_tiles, l1, bias_decay, lr,
              out, B, d, step, gscale, cnt_part=None, feat_count=None, b1=0.9, b2=0.999, eps=1e-8,
              update=True, step_dev=None, defer_step=False):
    """Loss bookkeeping + bias Adam.  ``colpart`` [G, tm, n] holds partial sums of the bias
    gradient; ``gscale`` converts their sum to dL/db.  ``defer_step``: leave the device step
    counter alone (bias Adam uses ``*step_dev + 1``; the caller advances it) -- for running
    concurrently with a row-Adam that reads the same counter."""
    G, n = b.shape
    bc1 = 1.0 - b1 ** max(step, 1)
    bc2 = 1.0 - b2 ** max(step, 1)
    rc = _lib.lib().sc_bias_loss(
        G, _lib.ptr(b), _lib.ptr(m), _lib.ptr(v), _lib.ptr(colpart), tm, _lib.ptr(enc_part),
        enc_tiles, _lib.ptr(dec_part), dec_tiles, _lib.ptr(cnt_part), _lib.ptr(feat_count),
        _lib.ptr(l1), _lib.ptr(bias_decay), _lib.ptr(lr), _lib.ptr(out), n, B, d, float(gscale), b1, b2, eps,
        bc1, bc2, int(update), _lib.ptr(step_dev), _lib.stream_handle(), int(bool(defer_step)),
        int(cnt_part.shape[1]) if cnt_part is not None and cnt_part.dim() == 3 else 0,
    )
    _lib.check(rc, "sc_bias_loss")


TICKET_INTS = (1 + 64) * 32  # csrc/adam.hip: top + TK_SUB sub-counters, one 128-byte line each


def step_tail(sets, lr, b1, b2, eps, step_dev, bias, bias_m, bias_v, colpart, enc_part, dec_part, l1, bias_decay,
              out, B, gscale, bsq, ticket, cnt_part=None, feat_count=None, gather=None, nsplit=1, gstride=0,
              live=None, row0=None, live_host=None):
    """The end of a single-device step as ONE launch (csrc/adam.hip ``step_tail_kernel``): row Adam over
    ``sets`` (as ``adam_rows``), the loss terms into ``out`` [G, 6], bias Adam (gradient = ``gscale``
    x the column sums of ``colpart`` [G, tm, n]), feature on-counts when ``cnt_part`` /
    ``feat_count`` are given (``cnt_part`` [G, cnt_tm, n] may have its own slot count: a data-parallel
    bias gradient arrives already reduced, ``colpart`` = g_bias [G, 1, n] with ``gscale`` 1), and -- with ``gather`` = (ring buffer [N, d], perm int64, ep0 int32 [1],
    out [rows, d]) -- the NEXT step's batch fetch.  The device step counter ``step_dev`` is read by
    every block and advanced by the last one.  ``bsq`` [2, G, n/32] fp32 holds the b^2 partial sums
    of the current bias at index ``step & 1`` (``bias_sq_parts``); the tail writes the other half.
    ``ticket``: ``TICKET_INTS`` zero-initialised int32 (completion counters; reset by the kernel).  ``nsplit`` / ``gstride``: each set's
    gradient is the first of ``nsplit`` split-K partial slabs (as ``adam_rows``).  ``live``: int32 [G] live
    row counts of a masked ensemble (rows past them are skipped, as ``adam_rows``; with ``live_host``, the
    same sizes as host ints, the row blocks cover only live rows).  ``row0``: the sets are
    [rows, d] views of rows [row0, row0 + rows) of the [G n, d] stacks (a ZeRO-1 shard)."""
    shp = tuple(sets[0]["p"].shape)
    d = shp[-1]
    nrows = sets[0]["p"].numel() // d
    G, n = bias.shape
    if row0 is not None:  # a row shard: check it, then treat it like the full stack below
        if len(shp) != 2 or row0 < 0 or row0 + shp[0] > G * n:
            raise ValueError(f"row shard [{shp}] at row {row0} is outside the [{G} x {n}] stack")
        shp = (G, n, d)
    gbf16 = sets[0]["g"].dtype == torch.bfloat16
    for s in sets:
        for k in ("p", "g", "m", "v"):
            t = s[k]
            want = torch.bfloat16 if (k == "g" and gbf16) else torch.float32
            if t.dtype != want or tuple(t.shape) != tuple(sets[0]["p"].shape) or not t.is_contiguous():
                raise ValueError(f"step_tail set tensor {k} must be contiguous {want} {shp}")
    if len(shp) != 3 or shp[0] != G or shp[1] != n or n % 32 or d % 256 or d > 1024:
        raise ValueError(f"step_tail needs [G, n, d] sets with n % 32 == 0, d in 256..1024 (got {shp}, bias {G}x{n})")
    if tuple(bsq.shape) != (2, G, n // 32) or bsq.dtype != torch.float32 or not bsq.is_contiguous():
        raise ValueError("bsq must be contiguous fp32 [2, G, n/32]")
    if ticket.dtype != torch.int32 or ticket.numel() < TICKET_INTS or step_dev is None:
        raise ValueError("ticket must be int32 and step_dev a device counter")
    tm = colpart.shape[1]
    cnt_tm = cnt_part.shape[1] if cnt_part is not None else tm
    if tuple(colpart.shape) != (G, tm, n) or (cnt_part is not None and tuple(cnt_part.shape) != (G, cnt_tm, n)):
        raise ValueError("colpart must be [G, tm, n] and cnt_part [G, cnt_tm, n]")
    gbuf = perm = ep0 = gout = None
    grows = row_bytes = nbuf = nperm = 0
    if gather is not None:
        gbuf, perm, ep0, gout = gather
        row_bytes = gbuf.shape[-1] * gbuf.element_size()
        if (row_bytes % 16 or gout.dtype != gbuf.dtype or gout.shape[-1] != gbuf.shape[-1] or not gout.is_contiguous()
                or perm.dtype != torch.int64 or ep0.dtype != torch.int32):
            raise ValueError("gather: contiguous rows of 16-byte multiples, int64 perm, int32 ep0")
        grows, nbuf, nperm = gout.shape[0], gbuf.shape[0], perm.numel()
    rows = (C.c_int * len(sets))(*[nrows for _ in sets])
    norm = (C.c_int * len(sets))(*[int(bool(s["norm"])) for s in sets])
    rc = _lib.lib().sc_step_tail(
        len(sets), _vp([s["p"] for s in sets]), _vp([s["g"] for s in sets]),
        _vp([s["m"] for s in sets]), _vp([s["v"] for s in sets]),
        _vp([s.get("shadow") for s in sets]), _vp([s.get("norms") for s in sets]),
        rows, norm, d, n, _lib.ptr(lr), b1, b2, eps, _lib.ptr(step_dev), int(gbf16),
        G, _lib.ptr(bias), _lib.ptr(bias_m), _lib.ptr(bias_v), _lib.ptr(colpart), tm, _lib.ptr(enc_part),
        enc_part.shape[1], _lib.ptr(dec_part), dec_part.shape[1], _lib.ptr(cnt_part), _lib.ptr(feat_count),
        _lib.ptr(l1), _lib.ptr(bias_decay), _lib.ptr(out), n, B, float(gscale), _lib.ptr(bsq), _lib.ptr(ticket),
        _lib.ptr(gbuf), nbuf, _lib.ptr(perm), nperm, _lib.ptr(ep0), _lib.ptr(gout), grows, row_bytes,
        int(nsplit), int(gstride), _lib.ptr(live), int(cnt_tm), int(row0 or 0),
        C.cast((C.c_int * len(live_host))(*[int(v) for v in live_host]), C.c_void_p)
        if (live_host is not None and live is not None) else None, _lib.stream_handle(),
    )
    _lib.check(rc, "sc_step_tail")


def topk_tail(p, g, m, v, shadow, norms, lr, b1, b2, eps, step_dev, row_se, mse, se_scale, ticket, gather=None):
    """The end of a top-k step as ONE launch (csrc/adam.hip ``sc_topk_tail``): row Adam with the norm
    Jacobian on the dictionary stack ``p`` [G, n, d] (as ``adam_rows``, bf16 shadow + row norms),
    ``mse[g] = se_scale * sum(row_se[g])`` (row_se [G, B] per-row squared errors), the NEXT step's batch
    fetch with ``gather`` = (ring buffer [N, d], perm int64, ep0 int32 [1], out [rows, d]), and the
    device step counter ``step_dev`` read by every block and advanced by the last one."""
    G, n, d = p.shape
    gbf16 = g.dtype == torch.bfloat16
    for name, t, want in (("p", p, torch.float32), ("m", m, torch.float32), ("v", v, torch.float32),
                          ("g", g, torch.bfloat16 if gbf16 else torch.float32)):
        if t.dtype != want or tuple(t.shape) != (G, n, d) or not t.is_contiguous():
            raise ValueError(f"topk_tail tensor {name} must be contiguous {want} {(G, n, d)}")
    if d % 256 or d > 1024:
        raise ValueError(f"topk_tail needs d in 256..1024, a multiple of 256 (got {d})")
    if shadow.dtype != torch.bfloat16 or shadow.numel() != G * n * d or norms.numel() != G * n:
        raise ValueError("shadow must be bf16 [G, n, d] and norms [G, n]")
    if (row_se.dtype != torch.float32 or row_se.dim() != 2 or row_se.shape[0] != G or not row_se.is_contiguous()
            or mse.dtype != torch.float32 or mse.numel() != G):
        raise ValueError("row_se must be contiguous fp32 [G, rows] and mse fp32 [G]")
    if ticket.dtype != torch.int32 or ticket.numel() < TICKET_INTS or step_dev is None:
        raise ValueError("ticket must be int32 and step_dev a device counter")
    gbuf = perm = ep0 = gout = None
    grows = row_bytes = nbuf = nperm = 0
    if gather is not None:
        gbuf, perm, ep0, gout = gather
        row_bytes = gbuf.shape[-1] * gbuf.element_size()
        if (row_bytes % 16 or gout.dtype != gbuf.dtype or gout.shape[-1] != gbuf.shape[-1] or not gout.is_contiguous()
                or perm.dtype != torch.int64 or ep0.dtype != torch.int32):
            raise ValueError("gather: contiguous rows of 16-byte multiples, int64 perm, int32 ep0")
        grows, nbuf, nperm = gout.shape[0], gbuf.shape[0], perm.numel()
    rc = _lib.lib().sc_topk_tail(
        _lib.ptr(p), _lib.ptr(g), _lib.ptr(m), _lib.ptr(v), _lib.ptr(shadow), _lib.ptr(norms), G, n, d,
        _lib.ptr(lr), b1, b2, eps, _lib.ptr(step_dev), int(gbf16), _lib.ptr(row_se), row_se.shape[1],
        float(se_scale), _lib.ptr(mse), _lib.ptr(ticket), _lib.ptr(gbuf), nbuf, _lib.ptr(perm), nperm,
        _lib.ptr(ep0), _lib.ptr(gout), grows, row_bytes, _lib.stream_handle(),
    )
    _lib.check(rc, "sc_topk_tail")


def bias_sq_parts(bias, bsq, parity: int):
    """bsq[parity] = per-32-column sums of bias^2 (what the step tail reads as |b|^2)."""
    G, n = bias.shape
    torch.sum(bias.view(G, n // 32, 32).square(), dim=-1, out=bsq[parity])
