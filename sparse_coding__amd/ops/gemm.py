"""Python front-end of the grouped MFMA GEMM (``csrc/sae_gemm.hip``).

Every function takes already-allocated output tensors so the training step
never allocates; shapes are checked on the host before launch (a mis-shaped
launch on MI355X can fault the whole node).

Notation: G = models in the ensemble, B = batch rows, d = activation width,
n = dictionary size.  bf16 tensors are passed as torch.bfloat16.
"""

from __future__ import annotations

import ctypes as C

import torch

from . import _lib

EPI_ENC, EPI_DEC, EPI_DC, EPI_F32, EPI_BF16, EPI_ENC_CNT, EPI_DC_MASK = 0, 1, 2, 3, 4, 6, 7
EPI_ENC_ACT, EPI_DC_ACT, EPI_ROWMAX = 8, 9, 10
# code activations of the ENC_ACT / DC_ACT epilogues
ACT_RELU, ACT_REVERSE, ACT_THRESHOLD = 0, 1, 2
TILE_M, TILE_N, TILE_K = 128, 128, 64

# Block shapes of the kernel (BK64 x 2-stage LDS-DMA ring for all of them):
#   0: automatic -- the largest shape that divides (M, N) and still launches >= 256 blocks
#   1: 128x128, 4 waves of 64x64        2: 256x128, 4 waves of 128x64
#   3: 256x256, 8 waves of 128x64 (one block per CU)
# Per-epilogue defaults come from measurements on MI355X (profiles/).
# Measured at B=2048, d=512, n=2048, G=8 (profiles/kernel_bench_r1_v6.jsonl): the fused
# epilogues are fastest on 128x128 blocks (two blocks per CU overlap one block's epilogue
# with the other's MFMA loop: enc 61 vs 84 us on 256x256), the plain fp32 weight-gradient
# GEMM (K = B = 2048) on 256x256 blocks (65 vs 74 us; 0.3311 vs 0.3460 ms per step) -- "auto"
# picks that.  A persistent 128x128 tile loop with a continuous LDS-DMA stream across tiles
# (bit-identical, not faster: two co-resident workgroups per CU already hide the same
# latencies) and Adam fused into the weight-gradient epilogue were measured and removed.
# Round 4, in-step A/B on one box (profiles/r4/cfg_ab/): the encoder and code-gradient epilogues on
# 128x128 blocks with the BK32 x 3-stage ring (cfg 13: 48 KB of LDS instead of 64, so one more
# workgroup co-resides per CU) -- 0.2932 / 0.2947 vs 0.3100 / 0.3088 ms per step with BK64 x 2
# (isolated kernel timings showed only ~1 us: the gain is in-step co-residency)
# Round 5 (profiles/r5/batch4/): the same BK32 x 3 ring with the software-pipelined K loop (cfg bit 4:
# 13 | 16 = 29; the next K-tile's fragments are read while the current tile's MFMAs run, three waves
# per SIMD kept) -- step median 0.2893 vs 0.2915 ms over 4 alternating runs each on one box.
# Round 6 (profiles/r6/w8/): 256x128 blocks of EIGHT 64x64 waves on the BK32 x 3 ring (cfg 14 = shape 2 |
# pipe 3; 72 KB, <= 128 VGPRs: two blocks / sixteen waves per CU) for the encoder and the bitmask code
# gradient (EPI_DC_MASK) -- 25 % fewer operand bytes per FLOP than 128x128 at the same per-wave tile: step 0.2873 vs
# 0.2926 ms (3 alternating runs each, same box; again 0.2869 vs 0.2918 on a second box).  Not for the
# counting encoder (its epilogue spills at 128 VGPRs: slower), the decoder (slower) or masked-ensemble
# launches (nactive / nact_k: they fall back to cfg 29 below).
_CFG_DEFAULT = {EPI_ENC: 14, EPI_DEC: 1, EPI_DC: 1, EPI_F32: 0, EPI_BF16: 0, EPI_ENC_CNT: 29,
                EPI_DC_MASK: 14, EPI_ENC_ACT: 1, EPI_DC_ACT: 1, EPI_ROWMAX: 1}
_CFG_FALLBACK = {14: 29}  # 256x128 eight-wave default -> the 128x128 pipelined BK32 x 3 ring (M % 256 != 0)
_CFG_OVERRIDE = None
# (epi, operand layout) -> cfg: overrides _CFG_DEFAULT for that layout only.  The bf16-out GEMMs of the
# top-k step (scores x D^T: layout 3; the two-segment dense weight gradient: layout 0) on the eight-wave
# 256x128 block: config 4 0.988-0.993 vs 1.012-1.015 ms/step (profiles/r6/w8/)
# The fp32 weight gradients (layout 0) too: headline 0.2822 vs 0.2833 ms median over 5 alternating runs
# (profiles/r6/wg14/).
_CFG_LAYOUT = {(EPI_BF16, 3): 14, (EPI_BF16, 0): 14, (EPI_F32, 0): 14}


def _env_cfgs():
    """``SC_GEMM_CFG="epi:cfg,..."`` (e.g. ``0:13,6:13,7:13``) overrides per-epilogue defaults, and
    ``epi/layout:cfg`` (e.g. ``4/3:29``) one operand layout of an epilogue only (bit 0: A K-major,
    bit 1: B K-major) -- for same-box A/B runs of whole steps (scripts/gemm_lab.py times the kernels
    in isolation)."""
    import os

    spec = os.environ.get("SC_GEMM_CFG", "").strip()
    for item in filter(None, spec.split(",")):
        key, cfg = item.split(":")
        if "/" in key:
            epi, layout = key.split("/")
            _CFG_LAYOUT[(int(epi), int(layout))] = int(cfg)
        else:
            _CFG_DEFAULT[int(key)] = int(cfg)


_env_cfgs()
SHAPES = {1: (128, 128), 2: (256, 128), 3: (256, 256)}
# cfg bits 2-3 select the K pipeline: 0 BK64 x 2-stage LDS ring (default), 1 BK32 x 4,
# 2 BK32 x 2 (smallest LDS footprint: most co-resident blocks), 3 BK32 x 3 (the
# alternatives exist for the step's epilogues and the weight-gradient layout only); bit 4: the
# software-pipelined K loop on the 128x128 BK32 rings.
PIPES = {0: (64, 2), 1: (32, 4), 2: (32, 2), 3: (32, 3)}


def set_config(epi: int, cfg: int):
    _CFG_DEFAULT[epi] = int(cfg)


class force_shape:
    """Context manager: run every GEMM with block shape ``cfg`` (tests / A-B timing)."""

    def __init__(self, cfg: int):
        self.cfg = int(cfg)

    def __enter__(self):
        global _CFG_OVERRIDE
        self._old, _CFG_OVERRIDE = _CFG_OVERRIDE, self.cfg
        return self

    def __exit__(self, *exc):
        global _CFG_OVERRIDE
        _CFG_OVERRIDE = self._old


def shape_fits(cfg: int, M: int, N: int) -> bool:
    bm, bn = SHAPES.get(int(cfg) & 3, (128, 128))
    return M % bm == 0 and N % bn == 0


def _op(t, ld, sg):
    return _lib.ScOperand(_lib.ptr(t), ld, sg)


def _need(cond, msg):
    if not cond:
        raise ValueError(msg)


def _bf16(t, name):
    _need(t.dtype == torch.bfloat16, f"{name} must be bfloat16, got {t.dtype}")
    _need(t.is_cuda, f"{name} must be on the GPU")
    _need(t.is_contiguous(), f"{name} must be contiguous")


def _launch(epi, layout, M, N, K1, K2, G, a_ops, b_ops, outs, alphas, ldc, sc, *,
            bias=None, sbias=0, nactive=None, aux=None, ldaux=0, saux=0, part=None,
            colpart=None, l1=None, l1_add_scale=0.0, dotpart=None, dc_tied=False, cfg=None,
            ksplit=1, split_stride=0, cmask=None, act=0, ascale=None, cmask2=None, rcol=None, nact_m=None,
            nact_k=None, nact_host=None):
    _need(M % TILE_M == 0 and N % TILE_N == 0, f"M={M}, N={N} must be multiples of 128")
    _need(K1 % TILE_K == 0 and K2 % TILE_K == 0, f"K={K1}+{K2} must be multiples of 64")
    if cfg is None:
        cfg = _CFG_OVERRIDE if _CFG_OVERRIDE is not None else _CFG_LAYOUT.get((epi, layout), _CFG_DEFAULT[epi])
        if _CFG_OVERRIDE is None and (((cfg & 3) and not shape_fits(cfg, M, N))
                                      or (cfg in _CFG_FALLBACK and (nactive is not None or nact_k is not None
                                                                    or nact_m is not None))):
            # a default whose block does not tile this problem; masked launches keep the 128x128 ring
            # (their compacted live tiles pack better in its three slots per CU: profiles/r6/w8/)
            cfg = 0 if epi == EPI_F32 else _CFG_FALLBACK.get(cfg, 1)  # (fp32 out: the automatic shape)
    cfg = int(cfg)
    _need((cfg & 3) == 0 or shape_fits(cfg, M, N), f"block shape {SHAPES.get(cfg & 3)} does not tile M={M}, N={N}")
    nprob = len(outs)
    A = (_lib.ScOperand * (2 * nprob))(*a_ops)
    Bo = (_lib.ScOperand * (2 * nprob))(*b_ops)
    Cp = (C.c_void_p * nprob)(*[_lib.ptr(o) for o in outs])
    al = (C.c_float * nprob)(*alphas)
    # host copy of a masked ensemble's live sizes: the launcher then launches only live tiles
    nh = (C.c_int * len(nact_host))(*[int(v) for v in nact_host]) if nact_host is not None else None
    rc = _lib.lib().sc_gemm(
        epi, layout, nprob, M, N, K1, K2, G, A, Bo, Cp, al, ldc, sc,
        _lib.ptr(bias), sbias, _lib.ptr(nactive), _lib.ptr(aux), ldaux, saux,
        _lib.ptr(part), _lib.ptr(colpart), _lib.ptr(l1), float(l1_add_scale),
        _lib.ptr(dotpart), int(bool(dc_tied)),
        cfg, int(ksplit), int(split_stride), _lib.ptr(cmask), int(act), _lib.ptr(ascale),
        _lib.ptr(cmask2), _lib.ptr(rcol), _lib.ptr(nact_m), _lib.ptr(nact_k),
        C.cast(nh, C.c_void_p) if nh is not None else None, _lib.stream_handle(),
    )
    _lib.check(rc, f"sc_gemm(epi={epi})")


def _x_stride(x, B, d, G):
    """x may be shared by every model ([B, d]) or per model ([G, B, d])."""
    if x.dim() == 2:
        _need(tuple(x.shape) == (B, d), f"x shape {tuple(x.shape)} != {(B, d)}")
        return 0
    _need(tuple(x.shape) == (G, B, d), f"x shape {tuple(x.shape)} != {(G, B, d)}")
    return B * d


def code_mask_shape(G, B, n):
    """Shape of the encoder's activity bitmask: one 64-bit word per lane per 64x64 block of the
    codes (csrc/sae_gemm_kernel.h, mask_bit)."""
    return (G, B // 64, n // 64, 64)


def encode_relu(x, w, bias, c_out, part, colpart=None, nactive=None, mask_out=None, act=ACT_RELU, ascale=None,
                mask2_out=None, live_host=None):
    """c[g] = relu(x[g] @ w[g]^T + bias[g]) with L1/L0 partials.

    ``act`` selects another code activation of the same GEMM:
    ``ACT_REVERSE`` c = 1[pre > 0] (pre - bias) (L1 partial = sum |c|, L0 = active count);
    ``ACT_THRESHOLD`` c = s2 thr(pre / s2) with ``ascale`` = s2 [G, n] fp32 and ``bias``
    the per-feature gain.

    x: [B, d] or [G, B, d] bf16; w: [G, n, d] bf16; bias: [G, n] fp32;
    c_out: [G, B, n] bf16; part: [G, (B/128)*(n/128), 2] fp32;
    colpart (optional): [G, B/128, n] fp32 per-feature on-counts;
    mask_out (optional): int64 ``code_mask_shape(G, B, n)``: the activity bitmask ``code_grad``
    can read instead of the codes.
    mask2_out (``ACT_THRESHOLD``): the same layout, 1 where the code is on the threshold's ramp
    (decided on the fp32 pre-activation; ``code_grad(mask2=...)`` reads it).
    live_host (with ``nactive``): the same live sizes as host ints -- only live tiles are then
    launched and nothing past a model's live size is written (``c_out`` / ``colpart`` / ``part``
    must hold zeros there, as the engine's zero-initialised buffers do); ``code_grad`` and
    ``weight_grads`` take it too.
    """
    G, n, d = w.shape
    B = c_out.shape[1]
    _bf16(x, "x"); _bf16(w, "w"); _bf16(c_out, "c_out")
    sx = _x_stride(x, B, d, G)
    _need(tuple(c_out.shape) == (G, B, n), "c_out shape")
    _need(tuple(bias.shape) == (G, n) and bias.dtype == torch.float32, "bias shape/dtype")
    _need(part.numel() >= G * (B // 128) * (n // 128) * 2, "part too small")
    if colpart is not None:
        _need(colpart.numel() >= G * (B // 128) * n, "colpart too small")
    if nactive is not None:
        _need(nactive.dtype == torch.int32 and nactive.numel() == G, "nactive must be int32[G]")
    if mask_out is not None:
        _need(mask_out.dtype == torch.int64 and tuple(mask_out.shape) == code_mask_shape(G, B, n)
              and mask_out.is_contiguous(), "mask_out must be contiguous int64 code_mask_shape(G, B, n)")
    if act == ACT_THRESHOLD:
        _need(ascale is not None and tuple(ascale.shape) == (G, n) and ascale.dtype == torch.float32
              and ascale.is_contiguous(), "threshold activation needs ascale fp32 [G, n]")
    if mask2_out is not None:
        _need(act == ACT_THRESHOLD and mask2_out.dtype == torch.int64
              and tuple(mask2_out.shape) == code_mask_shape(G, B, n) and mask2_out.is_contiguous(),
              "mask2_out: int64 code_mask_shape(G, B, n), threshold activation only")
    a = [_op(x, d, sx), _op(x, d, sx)]
    b = [_op(w, d, n * d), _op(w, d, n * d)]
    epi = EPI_ENC_ACT if act != ACT_RELU else (EPI_ENC_CNT if colpart is not None else EPI_ENC)
    _launch(epi, 3, B, n, d, 0, G, a, b, [c_out], [1.0], n, B * n,
            bias=bias, sbias=n, nactive=nactive, part=part, colpart=colpart, cmask=mask_out, act=act,
            ascale=ascale, cmask2=mask2_out, nact_host=live_host if nactive is not None else None)


def decode_residual(c, w_hat, x, r_out, part, rcol=None, nactive=None):
    """r[g] = c[g] @ w_hat[g] - x[g]  (bf16 out) with sum(r^2) partials.

    c: [G, B, n] bf16; w_hat: [G, n, d] bf16 (row-normalised dictionary);
    x: [B, d] or [G, B, d] bf16; r_out: [G, B, d] bf16; part: [G, (B/128)*(d/128)];
    rcol (optional): [G, B/128, d] fp32 column sums of the residual per 128-row tile, taken
    before the bf16 rounding.
    """
    G, B, n = c.shape
    d = w_hat.shape[2]
    _bf16(c, "c"); _bf16(w_hat, "w_hat"); _bf16(r_out, "r_out")
    sx = _x_stride(x, B, d, G)
    _need(tuple(w_hat.shape) == (G, n, d), "w_hat shape")
    _need(part.numel() >= G * (B // 128) * (d // 128), "part too small")
    if rcol is not None:
        _need(rcol.dtype == torch.float32 and rcol.numel() >= G * (B // 128) * d and rcol.is_contiguous(),
              "rcol must be fp32 [G, B/128, d]")
    a = [_op(c, n, B * n)] * 2
    b = [_op(w_hat, d, n * d)] * 2  # stored [K=n][N=d] -> N-major
    # nactive (masked ensembles): codes past a model's live size are zero -- skip those K-tiles
    _launch(EPI_DEC, 1, B, d, n, 0, G, a, b, [r_out], [1.0], d, B * d, nact_k=nactive,
            aux=x, ldaux=d, saux=sx, part=part, rcol=rcol)


def code_grad(r, w_hat, c, l1, dpre_out, colpart, dotpart=None, tied_bias=None, mask=None, act=ACT_RELU,
              ascale=None, mask2=None, nactive=None, live_host=None):
    """dpre_s[g] = 1[c>0] * (r[g] @ w_hat[g]^T + l1[g] * d / 2).

    dpre_s is the code gradient in units of the residual: dL/dpre = 2/(B d) * dpre_s.
    colpart receives per-row-tile column sums (bias gradient partials).  With ``dotpart``
    [G, B/128, n] the epilogue also accumulates the norm-Jacobian row dots
    <w_hat_j, dL/dw_hat_j> (in units of 2/(B d)); ``tied_bias`` ([G, n]) adds the tied
    dictionary's encoder-path term.  ``mask`` (the encoder's ``mask_out``) replaces the
    read of ``c`` by the 16x smaller activity bitmask when no dots are requested.

    With ``act`` (ACT_REVERSE / ACT_THRESHOLD, needs ``mask``): the code gradient of that
    activation.  Reverse: dpre_s = active * (r w^T + l1 d/2 sign(c)) and zero column sums
    (the bias gets no gradient through the codes).  Threshold (``ascale`` = s2): dpre_s =
    active * (r w^T + l1 d/2) thr', column sums = gain gradient, and ``dotpart`` receives
    the partials of sum_b dL/dc (thr - u thr') (x 2 s: the scale gradient).
    ``nactive`` (masked ensembles, the engine): column tiles wholly past a model's live size
    skip their MFMA work and leave ``dpre_out`` there unwritten (the weight gradient skips
    those rows); their bias-gradient partials are zeroed.
    """
    G, B, d = r.shape
    n = w_hat.shape[1]
    _bf16(r, "r"); _bf16(w_hat, "w_hat"); _bf16(c, "c"); _bf16(dpre_out, "dpre_out")
    _need(tuple(c.shape) == (G, B, n) and tuple(dpre_out.shape) == (G, B, n), "c/dpre shape")
    _need(l1.dtype == torch.float32 and l1.numel() == G, "l1 must be fp32[G]")
    _need(colpart.numel() >= G * (B // 128) * n, "colpart too small")
    a = [_op(r, d, B * d)] * 2
    b = [_op(w_hat, d, n * d)] * 2
    if dotpart is not None:
        _need(dotpart.numel() >= G * (B // 128) * n, "dotpart too small")
    if act != ACT_RELU:
        _need(mask is not None and mask.dtype == torch.int64 and tuple(mask.shape) == code_mask_shape(G, B, n),
              "activation code gradient needs the encoder's mask")
        if act == ACT_THRESHOLD:
            _need(ascale is not None and tuple(ascale.shape) == (G, n) and ascale.dtype == torch.float32
                  and ascale.is_contiguous(), "threshold activation needs ascale fp32 [G, n]")
        if mask2 is not None:
            _need(act == ACT_THRESHOLD and mask2.dtype == torch.int64
                  and tuple(mask2.shape) == code_mask_shape(G, B, n), "mask2 must match the encoder's mask2_out")
        _launch(EPI_DC_ACT, 3, B, n, d, 0, G, a, b, [dpre_out], [1.0], n, B * n,
                aux=c, ldaux=n, saux=B * n, colpart=colpart, l1=l1, l1_add_scale=d / 2.0,
                dotpart=dotpart, cmask=mask, act=act, ascale=ascale, sbias=n, cmask2=mask2, nactive=nactive,
                nact_host=live_host if nactive is not None else None)
        return
    if mask is not None and dotpart is None:
        _need(mask.dtype == torch.int64 and tuple(mask.shape) == code_mask_shape(G, B, n), "mask shape")
        _launch(EPI_DC_MASK, 3, B, n, d, 0, G, a, b, [dpre_out], [1.0], n, B * n,
                colpart=colpart, l1=l1, l1_add_scale=d / 2.0, cmask=mask, nactive=nactive,
                nact_host=live_host if nactive is not None else None)
        return
    _launch(EPI_DC, 3, B, n, d, 0, G, a, b, [dpre_out], [1.0], n, B * n,
            aux=c, ldaux=n, saux=B * n, colpart=colpart, l1=l1, l1_add_scale=d / 2.0,
            dotpart=dotpart, dc_tied=tied_bias is not None, bias=tied_bias, sbias=n)


def wgrad_split(G, n, d, K, nprob, live=None):
    """Split-K factor for the weight-gradient GEMM: 1 while the 256x256 grid already fills
    the 256 CUs; otherwise the smallest power of two that reaches 256 blocks and keeps
    >= 1024 rows of K per split (few models on a large gathered batch, e.g. one model per
    GPU with ensemble sharding at N = 8)."""
    if live is not None:  # masked ensembles launch only their live row tiles
        tiles = nprob * sum(min(max(1, n // 256), max(1, -(-int(s) // 256))) for s in live) * max(1, d // 256)
    else:
        tiles = nprob * G * max(1, n // 256) * max(1, d // 256)
    s = 1
    while tiles * s < 256 and K // (2 * s) >= 1024 and K % (2 * s * 64) == 0:
        s *= 2
    return s


def weight_grads(pairs, outs, alpha, ksplit=1, nactive=None, live_host=None, cfg=None):
    """out_i[g] = alpha * sum_segments A_s[g]^T @ B_s[g]   (reduction over batch rows).

    pairs: list (one per problem, 1 or 2 problems) of lists of (A, B) segments
    (1 or 2 segments, summed along K).  A: [G, Bk, n] bf16 (or [Bk, n] shared),
    B: [G, Bk, d] bf16 (or [Bk, d] shared).  outs: [G, n, d] fp32 (or all bf16), or with ``ksplit`` > 1
    [ksplit, G, n, d] partial slabs (their sum is the product; the Adam kernel sums them).
    ``cfg``: the block configuration (default: the launcher's layout default; split-K picks its own).
    """
    _need(1 <= len(pairs) == len(outs) <= 2, "1 or 2 problems")
    G, n, d = outs[0].shape[-3:]
    nseg = len(pairs[0])
    _need(all(len(p) == nseg for p in pairs) and 1 <= nseg <= 2, "segments")
    ks = []
    a_ops, b_ops = [], []
    for p in pairs:
        seg_a, seg_b = [], []
        for (A, Bm) in p:
            _bf16(A, "A"); _bf16(Bm, "B")
            Bk = A.shape[-2]
            sa = 0 if A.dim() == 2 else Bk * n
            sb = 0 if Bm.dim() == 2 else Bk * d
            _need(A.shape[-1] == n and Bm.shape[-1] == d and Bm.shape[-2] == Bk, "segment shapes")
            seg_a.append(_op(A, n, sa))
            seg_b.append(_op(Bm, d, sb))
        if nseg == 1:
            seg_a.append(seg_a[0]); seg_b.append(seg_b[0])
        a_ops += seg_a; b_ops += seg_b
        ks.append(tuple(x.shape[-2] for x, _ in p))
    _need(len(set(ks)) == 1, "all problems must share K segments")
    K1 = ks[0][0]
    K2 = ks[0][1] if nseg == 2 else 0
    want = (G, n, d) if ksplit == 1 else (ksplit, G, n, d)
    # bf16 outputs (every problem's): the plain bf16 epilogue -- Adam reads bf16 gradients
    odt = outs[0].dtype
    _need(odt in (torch.float32, torch.bfloat16), "out must be fp32 or bf16")
    for o in outs:
        _need(o.dtype == odt and tuple(o.shape) == want and o.is_contiguous(), f"out must be {want} {odt}")
    if ksplit > 1:
        cfg = 3 if shape_fits(3, n, d) else 1
    # nactive (masked ensembles): gradient rows past a model's live size are zero -- those tiles
    # skip their MFMAs and only write the zeros; with live_host they are not launched at all
    _launch(EPI_F32 if odt == torch.float32 else EPI_BF16, 0, n, d, K1, K2, G, a_ops, b_ops, list(outs),
            [alpha] * len(outs), d, n * d, cfg=cfg, ksplit=ksplit, split_stride=G * n * d, nact_m=nactive,
            nact_host=live_host if nactive is not None else None)


def rowmax_nt(a, b, alpha=1.0, cfg=None):
    """max_j alpha <a[g, i], b[g, j]> for every row i: [G, M, K] x [G, N, K] -> [G, M] fp32.

    The max-cosine-similarity reduction behind MMCS: the [M, N] similarity
    matrix stays in registers (EPI_ROWMAX partials per 64-column wave tile, a tiny max on
    the host side).  Any shapes: rows / columns / K are padded here (extra columns repeat
    b's first row, so they never change a max; K is zero-padded).
    """
    squeeze = a.dim() == 2
    if squeeze:
        a, b = a.unsqueeze(0), b.unsqueeze(0)
    G, M, K = a.shape
    N = b.shape[1]
    _need(b.shape[0] == G and b.shape[2] == K, f"shapes {tuple(a.shape)} x {tuple(b.shape)}")
    # 256x256 blocks (128x64 per wave) from 16M similarity entries on: 0.29 vs 0.37 ms at
    # 16k x 16k x 512, 3.72 vs 4.65 ms at 32k x 32k x 2048 (profiles/mmcs_bench_r1.jsonl)
    if cfg is None:
        cfg = 3 if M * N >= (1 << 24) else 1
    blk = 256 if cfg == 3 else 128
    Mp, Np, Kp = -(-M // blk) * blk, -(-N // blk) * blk, -(-K // 64) * 64
    bf = torch.bfloat16
    ap = torch.zeros(G, Mp, Kp, device=a.device, dtype=bf)
    ap[:, :M, :K] = a
    bp = torch.zeros(G, Np, Kp, device=a.device, dtype=bf)
    bp[:, :N, :K] = b
    if Np > N:
        bp[:, N:, :K] = b[:, :1]
    tiles = (Np // 128) * 2  # 128x128 blocks of two 64-column waves
    part = torch.empty(G, Mp, tiles, device=a.device, dtype=torch.float32)
    _launch(EPI_ROWMAX, 3, Mp, Np, Kp, 0, G, [_op(ap, Kp, Mp * Kp)] * 2, [_op(bp, Kp, Np * Kp)] * 2, [part],
            [float(alpha)], tiles, Mp * tiles, cfg=cfg)
    out = part.amax(dim=-1)[:, :M]
    return out[0] if squeeze else out


def matmul_nt(a, b, out, alpha=1.0):
    """out[g] = alpha * a[g] @ b[g]^T; a: [M, K] or [G, M, K]; b: [G, N, K]; out bf16/fp32 [G, M, N]."""
    G, N, K = b.shape
    M = a.shape[-2]
    _bf16(a, "a"); _bf16(b, "b")
    sa = 0 if a.dim() == 2 else M * K
    epi = EPI_F32 if out.dtype == torch.float32 else EPI_BF16
    _need(tuple(out.shape) == (G, M, N) and out.is_contiguous(), "out shape")
    _launch(epi, 3, M, N, K, 0, G, [_op(a, K, sa)] * 2, [_op(b, K, N * K)] * 2, [out], [alpha], N, M * N)


def matmul_nn(a, b, out, alpha=1.0):
    """out[g] = alpha * a[g] @ b[g]; a: [G, M, K] bf16, b: [G, K, N] bf16."""
    G, M, K = a.shape
    N = b.shape[2]
    _bf16(a, "a"); _bf16(b, "b")
    epi = EPI_F32 if out.dtype == torch.float32 else EPI_BF16
    _need(tuple(out.shape) == (G, M, N) and out.is_contiguous(), "out shape")
    _launch(epi, 1, M, N, K, 0, G, [_op(a, K, M * K)] * 2, [_op(b, N, K * N)] * 2, [out], [alpha], N, M * N)


def matmul_tn(a, b, out, alpha=1.0):
    """out[g] = alpha * a[g]^T @ b[g]; a: [G, K, M], b: [G, K, N] bf16 (reduction over rows)."""
    G, K, M = a.shape
    N = b.shape[2]
    _bf16(a, "a"); _bf16(b, "b")
    epi = EPI_F32 if out.dtype == torch.float32 else EPI_BF16
    _need(tuple(out.shape) == (G, M, N) and out.is_contiguous(), "out shape")
    _launch(epi, 0, M, N, K, 0, G, [_op(a, M, K * M)] * 2, [_op(b, N, K * N)] * 2, [out], [alpha], N, M * N)
