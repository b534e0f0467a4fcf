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
            if t.dtype != want or tuple(t.shape) != shp or not t.is_contiguous():
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
    )
    _lib.check(rc, "sc_bias_loss")
