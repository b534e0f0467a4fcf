"""``FusedSAEEnsemble``: the MI355X training engine for SAE ensembles.

One training step for ALL models of an ensemble is six kernel launches (the
reference runs ``vmap(grad(loss))`` + ``vmap(adam.update)``,
``autoencoders/ensemble.py:175-193``, i.e. dozens of eager ops):

1. ``encode_relu``     c = relu(x W_e^T + b)          (grouped MFMA GEMM, L1/L0 epilogue)
2. ``decode_residual`` R = c W_hat - x                (MFMA, sum R^2 epilogue)
3. ``code_grad``       dpre = 1[c>0](R W_hat^T + l d/2) (MFMA, bias-grad column partials)
4. ``weight_grads``    dW_hat = c^T R, dW_e = dpre^T x (two problems, one launch)
5. ``adam_rows``       norm-Jacobian + Adam + bf16 shadow for decoder and encoder
6. ``bias_loss``       reduce partials -> losses, Adam on the bias

State layout (per device): fp32 masters ``[G, n, d]``; Adam moments; bf16
shadows the GEMMs read (decoder shadow already row-normalised, so no kernel
ever recomputes norms); per-model hyper-parameters as device vectors
(``l1_alpha``, ``bias_decay``, ``lr``).  Nothing allocates inside ``step``.

Supported kinds: ``untied`` (FunctionalSAE / FunctionalMaskedSAE / FunctionalFista's
SAE loss) and ``tied`` (FunctionalTiedSAE with identity centering /
FunctionalMaskedTiedSAE), plus the tied activation variants ``reverse``
(FunctionalReverseSAE, codes 1[pre > 0](pre - b)) and ``threshold``
(FunctionalThresholdingSAE, learned scale / gain / centering), which run the
same kernels with the ENC_ACT / DC_ACT epilogues.  Masked models pass per-model
``dict_size``.
"""

from __future__ import annotations

import os

from typing import Dict, List, Optional, Sequence

import torch

from ..ops import adam as adam_ops
from ..ops import gemm as gemm_ops


# engine kind -> code activation of the encoder / code-gradient epilogues
_ACTS = {"untied": gemm_ops.ACT_RELU, "tied": gemm_ops.ACT_RELU, "reverse": gemm_ops.ACT_REVERSE,
         "threshold": gemm_ops.ACT_THRESHOLD}


def _upload(g, device):
    """Upload a freshly captured graph so its first replay does not pay the upload inline."""
    from ..ops import _lib

    with torch.cuda.device(device):
        _lib.upload_graph(g, device)


def _stack(models, key, which=0, device=None):
    return torch.stack([m[which][key].detach().float() for m in models]).to(device).contiguous()


class FusedSAEEnsemble:
    """Fused HIP training engine; API mirrors ``FunctionalEnsemble``."""

    def __init__(self, models, sig, lr=1e-3, batch_size=256, device="cuda", betas=(0.9, 0.999),
                 eps=1e-8, track_feature_counts=True, kind: Optional[str] = None,
                 count_every: int = 8, wgrad_split="auto", grad_dtype: Optional[str] = None):
        self.sig = sig
        self.kind = kind or getattr(sig, "fused_kind", None)
        # FunctionalTiedCenteredSAE (sae_ensemble.py:162-228): the tied kernels on x - center
        # with a learned center vector (updated by a small extra Adam step)
        self.learned_center = self.kind == "tied_centered"
        if self.learned_center:
            self.kind = "tied"
        if self.kind not in _ACTS:
            raise ValueError(f"signature {sig} has no fused implementation")
        # code activation of the encoder / code-gradient epilogues: reverse and threshold
        # SAEs are tied dictionaries with another activation (sae_ensemble.py:230-303, 445-501)
        self.act = _ACTS[self.kind]
        # the per-feature vector that plays the encoder bias (threshold SAEs: the gain)
        self._bkey = "activation_gain" if self.kind == "threshold" else "encoder_bias"
        self.device = torch.device(device)
        self.n_models = G = len(models)
        self.batch_size = B = int(batch_size)
        p0, b0 = models[0]
        self.n, self.d = p0["encoder"].shape
        n, d = self.n, self.d
        if B % 128 or n % 128 or d % 256:
            raise ValueError(f"fused path needs B%128==0, n%128==0, d%256==0 (got B={B}, n={n}, d={d})")
        # Tied SAEs may carry a fixed affine centering x_c = ((x - t) R^T) * s per model
        # (reference sae_ensemble.py:126-131).  Non-identity centering runs as one extra
        # grouped GEMM (x R^T) plus an elementwise pass into a per-model x_c buffer; every
        # later kernel then reads x_c (per-model operand stride).
        self.centering = None
        if self.kind == "tied" and "center_rot" in b0:
            eye = torch.eye(d)
            ident = all(torch.equal(m[1]["center_rot"].detach().float().cpu(), eye)
                        and not bool(m[1]["center_trans"].detach().any())
                        and bool((m[1]["center_scale"].detach() == 1).all()) for m in models)
            if not ident:
                rot = torch.stack([m[1]["center_rot"].detach().float() for m in models]).to(device)
                trans = torch.stack([m[1]["center_trans"].detach().float() for m in models]).to(device)
                scale = torch.stack([m[1]["center_scale"].detach().float() for m in models]).to(device)
                self.centering = {"rot": rot.to(torch.bfloat16).contiguous(),
                                  "tR": torch.bmm(trans.unsqueeze(1), rot.transpose(1, 2)),  # [G, 1, d]
                                  "scale": scale.unsqueeze(1).contiguous()}
        dev = self.device
        self.models_meta = [{k: v for k, v in m[1].items()} for m in models]
        self.betas, self.eps = betas, eps
        self.step_count = 0  # host mirror of the device counter below
        self.step_dev = torch.zeros(1, dtype=torch.int32, device=dev)  # completed Adam steps
        self.use_graph = False
        self._graph = None
        self._source = None  # in-graph batch source (attach_source)
        self._counted = False

        # ----- parameters (fp32 masters) and Adam state
        self.params: Dict[str, torch.Tensor] = {"encoder": _stack(models, "encoder", 0, dev),
                                                self._bkey: _stack(models, self._bkey, 0, dev)}
        if self.kind == "untied":
            self.params["decoder"] = _stack(models, "decoder", 0, dev)
        if self.kind == "threshold":
            # learned per-feature scale s (codes scale with s^2) and input centering vector
            self.params["activation_scale"] = _stack(models, "activation_scale", 0, dev)
            self.params["centering"] = _stack(models, "centering", 0, dev)
        if self.learned_center:
            self.params["center"] = _stack(models, "center", 0, dev)
        self.m = {k: torch.zeros_like(v) for k, v in self.params.items()}
        self.v = {k: torch.zeros_like(v) for k, v in self.params.items()}
        # ----- per-model hyper-parameters as device vectors
        self.l1 = torch.tensor([float(m[1]["l1_alpha"]) for m in models], device=dev, dtype=torch.float32)
        self.bias_decay = torch.tensor([float(m[1].get("bias_decay", 0.0)) for m in models], device=dev,
                                       dtype=torch.float32)
        lrs = lr if isinstance(lr, (list, tuple)) else [lr] * G
        self.lr = torch.tensor([float(x) for x in lrs], device=dev, dtype=torch.float32)
        self.nactive = None
        self._live = None  # host copy of the live sizes: masked launches cover only live tiles
        if "dict_size" in b0:
            self._live = [int(m[1]["dict_size"]) for m in models]
            self.nactive = torch.tensor(self._live, device=dev, dtype=torch.int32)

        # ----- bf16 shadows read by the GEMMs
        bf = torch.bfloat16
        self.enc_shadow = torch.empty(G, n, d, device=dev, dtype=bf)
        self.dec_shadow = torch.empty(G, n, d, device=dev, dtype=bf) if self.kind == "untied" else self.enc_shadow
        self.norms = torch.ones(G, n, device=dev)  # row norms of the normalised dictionary
        self.refresh_shadows()

        # ----- workspaces
        tm = B // 128
        # masked ensembles: the compacted launches never write past a model's live size, so the
        # buffers read there (codes, gradients) start, and stay, zero
        alloc = torch.zeros if self.nactive is not None else torch.empty
        self.c = alloc(G, B, n, device=dev, dtype=bf)
        self.r = torch.empty(G, B, d, device=dev, dtype=bf)
        # (masked: the wgrad GEMM's 256-row tiles read dpre columns past a model's live size that
        # the compacted 128-column code-gradient launch never writes -- they must read zero)
        self.dpre = alloc(G, B, n, device=dev, dtype=bf)
        # activity bitmask of c written by the encoder epilogue, read by the code-gradient
        # epilogue instead of c itself (1/16 of the bytes)
        self.cmask = torch.empty(gemm_ops.code_mask_shape(G, B, n), device=dev, dtype=torch.int64)
        # threshold SAEs: second bitmask, 1 on the activation's ramp (decided on the fp32
        # pre-activation in the encoder epilogue, read by the code gradient)
        self.cmask2 = torch.empty_like(self.cmask) if self.kind == "threshold" else None
        # gradient buffers; the last-produced weight gradient shares one flat buffer with the
        # reduced bias gradient so data-parallel runs all-reduce both with a single collective
        if self.kind == "untied":
            # one allocation [g_dec | g_enc | g_bias]: data-parallel runs can reduce all of a
            # chunk's gradients with one collective (grad_all) or in two ([g_dec], [g_enc|g_bias])
            self.grad_all = alloc(2 * G * n * d + G * n, device=dev, dtype=torch.float32)
            self.g_dec = self.grad_all[: G * n * d].view(G, n, d)
            self._g_flat = self.grad_all[G * n * d:]
            self.g_enc = self._g_flat[: G * n * d].view(G, n, d)
        else:
            # threshold / learned-centering SAEs append their small extra gradient sources (raw
            # column sums, scaled by alpha at the update) so data-parallel runs reduce them in
            # the same collective: [g_dec | g_bias | code-grad column sums | scale sums | R sums]
            self._n_extra = 0
            if self.kind == "threshold" or self.learned_center:
                self._n_extra = G * n + (G * n if self.kind == "threshold" else 0) + (G * d if self.learned_center else 0)
            self._g_flat = alloc(G * n * d + G * n + self._n_extra, device=dev, dtype=torch.float32)
            self.grad_all = self._g_flat
            self.g_dec = self._g_flat[: G * n * d].view(G, n, d)
            self.g_enc = None
        self.g_bias = self._g_flat[G * n * d: G * n * d + G * n].view(G, 1, n)
        self._x_gsum = self._x_dsum = self._x_rsum = None
        if getattr(self, "_n_extra", 0):
            off = G * n * d + G * n
            self._x_gsum = self._g_flat[off: off + G * n].view(G, n)
            off += G * n
            if self.kind == "threshold":
                self._x_dsum = self._g_flat[off: off + G * n].view(G, n)
                off += G * n
            if self.learned_center:
                self._x_rsum = self._g_flat[off: off + G * d].view(G, d)
        # Split-K of the single-device weight-gradient GEMM: with few models on a large
        # batch (ensemble sharding gives each GPU G/N models on N*B rows) the 256x256 grid
        # has fewer blocks than CUs, so the K = B reduction is split over blocks and the
        # Adam kernel sums the partial slabs.  (Data-parallel paths use the flat buffers.)
        nprob = 2 if self.kind == "untied" else 1
        kdim = B if self.kind == "untied" else 2 * B
        # (a code gradient fused into the encoder weight gradient, so dpre never reaches HBM, was
        # measured slower at d = 512 -- 127 vs 49 + ~33 us, per-CU operand feed -- and lives in
        # scripts/lab/sae_dcw.hip with its numbers in profiles/r4/dcw/README.md)
        self.wsplit = (gemm_ops.wgrad_split(G, n, d, kdim, nprob, live=self._live) if wgrad_split == "auto"
                       else int(wgrad_split))
        self.g_parts = (alloc(nprob, self.wsplit, G, n, d, device=dev, dtype=torch.float32)
                        if self.wsplit > 1 else None)
        self._g_from_parts = False
        # bf16 weight gradients for the single-device step (``grad_dtype='bf16'``): the
        # weight-gradient GEMM's bf16 epilogue and Adam's bf16-gradient loads
        # halve the gradient's HBM round trip; masters, moments and the update stay fp32.
        # Data-parallel paths keep the fp32 flat buffers (their all-reduce reads those).
        gdt = grad_dtype or "fp32"
        if gdt not in ("fp32", "bf16"):
            raise ValueError(f"grad_dtype must be 'fp32' or 'bf16', got {gdt!r}")
        self.g_bf = (alloc(nprob, G, n, d, device=dev, dtype=bf)
                     if gdt == "bf16" and self.wsplit == 1 else None)
        self._g_from_bf = False
        self.grad_scale = 1.0  # data parallel: 1 / world_size (gradients are then summed)
        slots = tm
        self.enc_part = torch.zeros(G, tm * (n // 128), 2, device=dev)
        self.dec_part = torch.zeros(G, tm * (d // 128), device=dev)
        self.colpart = torch.zeros(G, slots, n, device=dev)
        self.track_feature_counts = track_feature_counts
        # per-feature activation counts are sampled every `count_every` steps (the column
        # reduction costs ~15% of the encoder GEMM); `rows_seen` counts only sampled rows
        self.count_every = max(1, int(count_every))
        self.cnt_part = torch.zeros(G, slots, n, device=dev) if track_feature_counts else None
        self.feature_counts = torch.zeros(G, n, device=dev) if track_feature_counts else None
        self.rows_seen = 0
        self.out = torch.zeros(G, 6, device=dev)
        # fused step tail (csrc/adam.hip step_tail_kernel: row Adam + loss terms + bias Adam + the next
        # step's batch gather in ONE launch) for the plain untied / tied single-device step; it keeps
        # per-32-column b^2 partial sums (parity-double-buffered by the step counter) for |b|
        self._tail_ok = (self.kind in ("untied", "tied") and self.act == gemm_ops.ACT_RELU and not self.learned_center
                         and n % 32 == 0 and d <= 1024
                         and os.environ.get("SC_FUSED_TAIL", "1") not in ("", "0"))
        self._bsq = torch.zeros(2, G, n // 32, device=dev) if self._tail_ok else None
        self._ticket = torch.zeros(adam_ops.TICKET_INTS, device=dev, dtype=torch.int32) if self._tail_ok else None
        self._bsq_dirty = True
        # threshold SAEs: per-feature partial sums of the code gradient on the activation's ramp
        # (the scale gradient's source, written by the code-gradient epilogue)
        self.dotpart = torch.zeros(G, tm, n, device=dev) if self.kind == "threshold" else None
        self.x_static = torch.zeros(B, d, device=dev, dtype=bf)  # graph input buffer
        self._static_inputs = [self.x_static]
        if self.centering is not None or self.kind == "threshold" or self.learned_center:
            self._xr = torch.empty(G, B, d, device=dev)              # x R^T (fp32)
            self.x_c = torch.empty(G, B, d, device=dev, dtype=bf)    # centred input per model
        if self.kind == "threshold" or self.learned_center:
            self.s2 = torch.empty(G, n, device=dev)                  # s^2 read by the epilogues
            self._gsum = torch.empty(G, n, device=dev)
        # learned centering: fp32 column sums of the residual from the decoder epilogue (the
        # center gradient's direct term, taken before the bf16 rounding of R)
        self.rcol = torch.zeros(G, tm, d, device=dev) if self.learned_center else None

    def use_flat_grads(self):
        """Write the weight gradients straight into the fp32 flat buffer (``grad_all``): no split-K
        slabs, no bf16 gradient copy.  Data-parallel paths reduce that buffer, so they call this on
        every engine they wrap (an engine built with ``wgrad_split='auto'`` may have picked a split
        for its shape, e.g. 4 models on 2048 rows)."""
        self.wsplit = 1
        self.g_parts = None
        self.g_bf = None
        self._g_from_parts = self._g_from_bf = False
        return self

    # ------------------------------------------------------------------ helpers
    def _refresh_bsq(self):
        """The fused tail's b^2 partials of the current bias (after any update outside the tail)."""
        if self._bsq is not None:
            adam_ops.bias_sq_parts(self.params[self._bkey], self._bsq, self.step_count & 1)
        self._bsq_dirty = False

    def _tail_ready(self):
        if getattr(self, "_bsq_dirty", False) and self._bsq is not None:
            self._refresh_bsq()

    def refresh_shadows(self):
        """Rebuild the bf16 shadows from the fp32 masters (after any out-of-band edit)."""
        self._bsq_dirty = True
        if self.kind == "untied":
            adam_ops.shadow_rows(self.params["encoder"], self.enc_shadow, normalize=False)
            adam_ops.shadow_rows(self.params["decoder"], self.dec_shadow, self.norms, normalize=True)
        else:
            adam_ops.shadow_rows(self.params["encoder"], self.enc_shadow, self.norms, normalize=True)

    def refresh_decoder_shadow(self):
        """Rebuild only the decoder's bf16 shadow and row norms (untied SAEs; after an out-of-band edit
        of the decoder alone, e.g. the FISTA basis update) -- the encoder shadow is left as it is."""
        if self.kind != "untied":
            self.refresh_shadows()
            return
        adam_ops.shadow_rows(self.params["decoder"], self.dec_shadow, self.norms, normalize=True)

    def prepare(self, x):
        """The kernels' input: ``x`` itself, or its per-model centred copy for tied SAEs
        with non-identity centering (threshold SAEs: x - centering, learned)."""
        if self.kind == "threshold":
            self._center_rows(x, self.params["centering"])
            torch.mul(self.params["activation_scale"], self.params["activation_scale"], out=self.s2)
            return self.x_c
        if self.learned_center:
            self._center_rows(x, self.params["center"])
            return self.x_c
        if self.centering is None:
            return x
        c = self.centering
        gemm_ops.matmul_nt(x, c["rot"], self._xr)
        torch.sub(self._xr, c["tR"], out=self._xr)
        self._xr.mul_(c["scale"])
        self.x_c.copy_(self._xr)
        return self.x_c

    def _center_rows(self, x, c):
        """x_c[g] = bf16(x - c[g]) in one elementwise kernel (csrc/elementwise.hip)."""
        from ..ops import _lib

        G, B, d = self.x_c.shape
        if x.dtype != torch.bfloat16 or tuple(x.shape) != (B, d) or not x.is_contiguous():
            raise ValueError("centred input needs the contiguous bf16 [B, d] batch")
        rc = _lib.lib().sc_center_rows(_lib.ptr(x), _lib.ptr(c.contiguous()), _lib.ptr(self.x_c), G, B, d,
                                       _lib.stream_handle())
        _lib.check(rc, "sc_center_rows")

    def _x_bf16(self, batch):
        if batch.dtype != torch.bfloat16:
            batch = batch.to(torch.bfloat16)
        if batch.device != self.device:
            batch = batch.to(self.device, non_blocking=True)
        return batch.contiguous()

    # ------------------------------------------------------------------ forward/backward
    def _counting(self):
        return self.track_feature_counts and (self.step_count % self.count_every == 0)

    def forward(self, x, count=None, target=None):
        """Kernels 1-3: codes (+L1/L0), residual (+MSE), code gradient (+bias-grad partials).
        ``target``: the reconstruction target when it differs from the encoder input ``x``
        (threshold SAEs reconstruct the uncentred batch)."""
        if x.shape[-2] != self.batch_size:
            raise ValueError(f"batch has {x.shape[-2]} rows, engine was built for {self.batch_size}")
        count = self._counting() if count is None else count
        self._counted = count
        ascale = self.s2 if self.kind == "threshold" else None
        gemm_ops.encode_relu(x, self.enc_shadow, self.params[self._bkey], self.c, self.enc_part,
                             self.cnt_part if count else None, self.nactive, mask_out=self.cmask,
                             act=self.act, ascale=ascale, mask2_out=self.cmask2, live_host=self._live)
        gemm_ops.decode_residual(self.c, self.dec_shadow, x if target is None else target, self.r, self.dec_part,
                                 rcol=self.rcol, nactive=self.nactive)
        if self.act:
            gemm_ops.code_grad(self.r, self.dec_shadow, self.c, self.l1, self.dpre, self.colpart,
                               dotpart=self.dotpart if self.kind == "threshold" else None, mask=self.cmask,
                               act=self.act, ascale=ascale, mask2=self.cmask2, nactive=self.nactive,
                               live_host=self._live)
            return
        gemm_ops.code_grad(self.r, self.dec_shadow, self.c, self.l1, self.dpre, self.colpart,
                           mask=self.cmask, nactive=self.nactive, live_host=self._live)

    @property
    def _alpha(self):
        return 2.0 * self.grad_scale / (self.batch_size * self.d)

    def wgrad_first(self, x):
        """Untied: dW_hat = c^T R (decoder).  Tied: the whole dictionary gradient + bias grad."""
        self._g_from_parts = self._g_from_bf = False
        if self.kind == "untied":
            gemm_ops.weight_grads([[(self.c, self.r)]], [self.g_dec], self._alpha, nactive=self.nactive,
                                  live_host=self._live)
        else:
            gemm_ops.weight_grads([[(self.c, self.r), (self.dpre, x)]], [self.g_dec], self._alpha,
                                  nactive=self.nactive, live_host=self._live)
            self._reduce_bias_grad()

    def wgrad_second(self, x, reduce_bias=True):
        """Untied: dW_e = dpre^T x (encoder) + bias grad.  Tied: nothing."""
        if self.kind == "untied":
            self._enc_wgrad(x)
            if reduce_bias:
                self._reduce_bias_grad()

    def _enc_wgrad(self, x):
        """g_enc = alpha dpre^T x from the dpre the code-gradient GEMM wrote."""
        gemm_ops.weight_grads([[(self.dpre, x)]], [self.g_enc], self._alpha, nactive=self.nactive,
                              live_host=self._live)

    def _reduce_bias_grad(self):
        torch.sum(self.colpart, dim=1, keepdim=True, out=self.g_bias)
        self.g_bias.mul_(self._alpha)
        if self._x_gsum is not None:  # raw sums for the scale / centering updates (reduced with g_bias)
            torch.sum(self.colpart, dim=1, out=self._x_gsum)
            if self._x_dsum is not None:
                torch.sum(self.dotpart, dim=1, out=self._x_dsum)
            if self._x_rsum is not None:
                torch.sum(self.rcol, dim=1, out=self._x_rsum)

    def forward_backward(self, x):
        """Kernels 1-4 for the single-device step (both weight gradients in one launch)."""
        self.forward(x)
        self.backward_weights(x)

    def backward_weights(self, x):
        split = self.g_parts is not None
        self._g_from_parts = split
        self._g_from_bf = gbf = self.g_bf is not None
        if self.kind == "untied":
            outs = ([self.g_parts[0], self.g_parts[1]] if split else
                    [self.g_bf[0], self.g_bf[1]] if gbf else [self.g_dec, self.g_enc])
            gemm_ops.weight_grads([[(self.c, self.r)], [(self.dpre, x)]], outs, self._alpha, ksplit=self.wsplit,
                                  nactive=self.nactive, live_host=self._live)
        else:
            outs = [self.g_parts[0]] if split else [self.g_bf[0]] if gbf else [self.g_dec]
            gemm_ops.weight_grads([[(self.c, self.r), (self.dpre, x)]], outs, self._alpha, ksplit=self.wsplit,
                                  nactive=self.nactive, live_host=self._live)

    def _adam_sets(self):
        parts = self._g_from_parts
        gbf = self._g_from_bf
        g_dec = self.g_parts[0, 0] if parts else self.g_bf[0] if gbf else self.g_dec
        if self.kind == "untied":
            g_enc = self.g_parts[1, 0] if parts else self.g_bf[1] if gbf else self.g_enc
            return [dict(p=self.params["decoder"], g=g_dec, m=self.m["decoder"], v=self.v["decoder"],
                         shadow=self.dec_shadow, norms=self.norms, norm=True),
                    dict(p=self.params["encoder"], g=g_enc, m=self.m["encoder"], v=self.v["encoder"],
                         shadow=self.enc_shadow, norm=False)]
        return [dict(p=self.params["encoder"], g=g_dec, m=self.m["encoder"], v=self.v["encoder"],
                     shadow=self.enc_shadow, norms=self.norms, norm=True)]

    def _adam_split_kw(self):
        if self._g_from_parts:
            return dict(nsplit=self.wsplit, gstride=self.n_models * self.n * self.d)
        return {}

    def adam_first(self, reduced: bool = True):
        """Dictionary Adam (decoder for untied SAEs).  Threshold / learned-centering SAEs first
        update their scale and centering vectors: those gradients read the dictionary and must
        see it BEFORE this step's update (reference: every gradient from the same parameters,
        vmap(grad), autoencoders/ensemble.py:119-123)."""
        if self.kind == "threshold" or self.learned_center:
            self._threshold_extra_adam(reduced=reduced)
        adam_ops.adam_rows(self._adam_sets()[:1], self.lr, self.step_count + 1, *self.betas, self.eps,
                           step_dev=self.step_dev, live=self.nactive)

    def adam_rows_all(self):
        """Row Adam on every dictionary set (data-parallel update after the reduction)."""
        adam_ops.adam_rows(self._adam_sets(), self.lr, self.step_count + 1, *self.betas, self.eps,
                           step_dev=self.step_dev, live=self.nactive)

    def adam_second(self, reduced_bias=True):
        """Encoder Adam (untied) and bias Adam + loss reduction (advances the step counter)."""
        if self.kind == "untied":
            adam_ops.adam_rows(self._adam_sets()[1:], self.lr, self.step_count + 1, *self.betas, self.eps,
                               step_dev=self.step_dev, live=self.nactive)
        self._bias_loss(update=True, reduced=reduced_bias)
        self._host_step()

    def apply_update(self):
        """Kernels 5-6: fused Adam on the weights, then bias Adam + loss reduction."""
        self._tail_ready()
        self._apply_update_kernels()
        self._host_step()

    def _apply_update_kernels(self, gather=None):
        if self._tail_ok:
            # one launch: row Adam + loss terms + bias Adam (+ the next step's batch gather), the
            # device step counter advanced by its last block
            adam_ops.step_tail(self._adam_sets(), self.lr, *self.betas, self.eps, self.step_dev,
                               self.params[self._bkey], self.m[self._bkey], self.v[self._bkey], self.colpart,
                               self.enc_part, self.dec_part, self.l1, self.bias_decay, self.out, self.batch_size,
                               self._alpha, self._bsq, self._ticket,
                               cnt_part=self.cnt_part if self._counted else None,
                               feat_count=self.feature_counts if self._counted else None, gather=gather,
                               live=self.nactive, live_host=self._live, **self._adam_split_kw())
            return
        # scale / centering first: their gradients read the pre-update dictionary (adam_first)
        if self.kind == "threshold" or self.learned_center:
            self._threshold_extra_adam()
        adam_ops.adam_rows(self._adam_sets(), self.lr, self.step_count + 1, *self.betas, self.eps,
                           step_dev=self.step_dev, live=self.nactive, **self._adam_split_kw())
        self._bias_loss(update=True, reduced=False)

    def _threshold_extra_adam(self, reduced: bool = False):
        """Scale and centering of the threshold SAE (small vectors; before the bias / loss
        kernel, which advances the device step counter):
        dL/ds = 2 s alpha sum(dotpart), dL/dcentering = -alpha (sum_b dL/dpre) W_hat.
        Learned-centering tied SAEs also reconstruct x - center, so their center gradient
        gains the direct residual term + alpha sum_b R.  ``reduced``: take the column sums
        from the (data-parallel all-reduced) gradient buffer instead of this rank's partials."""
        a = self._alpha
        if reduced:
            self._gsum.copy_(self._x_gsum)
        else:
            torch.sum(self.colpart, dim=1, out=self._gsum)
        if self.learned_center:
            # the two terms largely cancel (dense codes: the residual's component outside the
            # active atoms' span survives), so both come from fp32 data: the decoder epilogue's
            # fp32 column sums of R (before its bf16 rounding) and the fp32 normalised masters
            w_hat = self.params["encoder"] / self.norms.unsqueeze(-1)
            g_c = torch.bmm(self._gsum.unsqueeze(1), w_hat).squeeze(1) * (-a)
            g_c += (self._x_rsum if reduced else self.rcol.sum(dim=1)) * a
        else:
            g_c = torch.bmm(self._gsum.unsqueeze(1).to(torch.bfloat16), self.enc_shadow).squeeze(1).float() * (-a)
        self.last_center_grad = g_c  # (inspection / tests: the centering gradient of this step)
        if self.learned_center:
            upd = (("center", g_c),)
        else:
            s = self.params["activation_scale"]
            if reduced:
                self._gsum.copy_(self._x_dsum)
            else:
                torch.sum(self.dotpart, dim=1, out=self._gsum)
            g_s = self._gsum * s * (2.0 * a)
            upd = (("activation_scale", g_s), ("centering", g_c))
        b1, b2 = self.betas
        t = bc1 = bc2 = None
        for k, g in upd:
            p, m, v = self.params[k], self.m[k], self.v[k]
            X = p.shape[-1]
            if p.dim() == 2 and X % 256 == 0 and X <= 4096:
                # one row-Adam launch per vector set (rows = models, device step counter): the
                # torch form below is ~10 launches of tiny elementwise kernels per vector
                adam_ops.adam_rows([dict(p=p, g=g.contiguous(), m=m, v=v, shadow=None, norms=None, norm=False)],
                                   self.lr, self.step_count + 1, *self.betas, self.eps, rows_per_model=1,
                                   step_dev=self.step_dev)
                continue
            if t is None:
                t = self.step_dev.float() + 1.0
                bc1 = 1.0 - torch.pow(b1, t)
                bc2 = 1.0 - torch.pow(b2, t)
            m.mul_(b1).add_(g, alpha=1.0 - b1)
            v.mul_(b2).addcmul_(g, g, value=1.0 - b2)
            p.sub_(self.lr.unsqueeze(1) * (m / bc1) / ((v / bc2).sqrt() + self.eps))

    def _host_step(self):
        if self._counted:
            self.rows_seen += self.batch_size
        self.step_count += 1

    def _bias_loss(self, update, reduced, defer_step=False):
        G, B, n, d = self.n_models, self.batch_size, self.n, self.d
        if update:
            self._bsq_dirty = True  # (a bias update outside the fused tail)
        b1, b2 = self.betas
        if reduced:  # bias gradient already summed (and possibly all-reduced) into g_bias
            colpart, tm, gscale = self.g_bias, 1, 1.0
        else:
            colpart, tm, gscale = self.colpart, self.colpart.shape[1], self._alpha
        adam_ops.bias_loss(self.params[self._bkey], self.m[self._bkey], self.v[self._bkey],
                           colpart, tm, self.enc_part, self.enc_part.shape[1], self.dec_part,
                           self.dec_part.shape[1], self.l1, self.bias_decay, self.lr, self.out, B, d,
                           self.step_count + 1, gscale=gscale,
                           cnt_part=self.cnt_part if self._counted else None,
                           feat_count=self.feature_counts if self._counted else None,
                           b1=b1, b2=b2, eps=self.eps, update=update,
                           step_dev=self.step_dev, defer_step=defer_step)

    def step_batch(self, batch, expand_dims=True):
        """One Adam step of every model on ``batch [B, d]``; returns a device tensor [G, 6]:
        (loss, l_reconstruction, l_l1, l_bias_decay, mean L0, |b|).  Never synchronises."""
        self._tail_ready()
        if self.use_graph:
            for i, t in enumerate(self._static_inputs):
                if batch is t:
                    return self.step_static(i)
            self.x_static.copy_(batch, non_blocking=True)
            return self.step_static()
        x = self._x_bf16(batch)
        self._step_kernels(x)
        self._host_step()
        return self.out

    # ------------------------------------------------------------------ HIP graph
    def enable_graph(self, enabled: bool = True):
        """Capture the whole step (7 kernels) into one HIP graph; inputs go through
        ``x_static``.  Removes the per-launch host overhead (the step is launch-bound
        at small batch)."""
        self.use_graph = enabled
        if not enabled:
            self._graph = None
        return self

    def _step_kernels(self, x, count=None, gather=None, before_update=None):
        """All kernels of one step (captured as one HIP graph when enabled).  Side-stream
        variants of this sequence -- decoder Adam beside the encoder weight gradient, the loss /
        bias-Adam tail beside the weight gradient, Adam fused into the weight-gradient epilogue,
        a fused weight-gradient + Adam kernel -- all measured slower on MI355X and were removed
        (profiles/README.md)."""
        target = x if self.kind == "threshold" else None
        x = self.prepare(x)
        self.forward(x, count, target)
        self.backward_weights(x)
        if before_update is not None:  # e.g. a stream wait the update (its next-batch fetch) needs
            before_update()
        self._apply_update_kernels(gather if self._tail_ok else None)

    def add_static_input(self, t: torch.Tensor) -> int:
        """Register another persistent input buffer [B, d] bf16: ``step_batch(t)`` then replays
        a graph captured on ``t`` itself (no copy into ``x_static``; e.g. the two halves of a
        double-buffered batch prefetch).  Returns its index for ``step_static``."""
        if t.dtype != torch.bfloat16 or tuple(t.shape) != (self.batch_size, self.d) or not t.is_contiguous():
            raise ValueError("static inputs must be contiguous bf16 [batch_size, d]")
        self._static_inputs.append(t)
        self._graph = None  # recapture on next use
        return len(self._static_inputs) - 1

    def _capture(self):
        torch.cuda.synchronize(self.device)
        self._graph = {}
        for i, xin in enumerate(self._static_inputs):
            for count in (True, False):
                g = torch.cuda.CUDAGraph()
                # thread_local: RCCL's watchdog thread may query events of in-flight
                # collectives while this thread captures (ensemble-sharded runs)
                with torch.cuda.graph(g, capture_error_mode="thread_local"):
                    self._step_kernels(xin, count)
                _upload(g, self.device)
                self._graph[(count, i)] = g

    def attach_source(self, source):
        """Fetch each step's batch INSIDE the captured graph from ``source`` (e.g.
        ``DeviceRing.graph_source(batch_size)``, indexed by the device step counter); then call
        ``step_source()`` per step.  Removes the plain gather launch between graph replays
        (an ~9 us idle gap per step on MI355X, profiles/README.md)."""
        ring = getattr(source, "ring", None)
        if ring is not None and (ring.buf.dtype != self.x_static.dtype or ring.buf.shape[-1] != self.d
                                 or getattr(source, "B", self.batch_size) != self.batch_size):
            raise ValueError(f"source rows are {ring.buf.dtype} [*, {ring.buf.shape[-1]}] in batches of "
                             f"{getattr(source, 'B', '?')}; the engine takes {self.x_static.dtype} "
                             f"[{self.batch_size}, {self.d}]")
        self._source = source
        self._graph = None
        return self

    def _source_graph(self, pattern):
        if self._source is None:
            raise RuntimeError("attach_source() first")
        if self._graph is None:
            self._capture()
        key = ("src", tuple(pattern))
        g = self._graph.get(key)
        if g is None:
            torch.cuda.synchronize(self.device)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                # each step's batch: the first step's own gather kernel; later steps' rows are fetched by
                # the previous step's fused tail (one launch fewer per step) when the source allows it
                nxt = self._source.tail_gather(self.x_static) if (self._tail_ok and hasattr(self._source, "tail_gather")) else None
                for i, count in enumerate(pattern):
                    if i == 0 or nxt is None:
                        self._source.gather(self.x_static, self.step_dev)
                    self._step_kernels(self.x_static, count, gather=nxt if i + 1 < len(pattern) else None)
            _upload(g, self.device)
            self._graph[key] = g
        return g

    def prime_source(self, steps: Optional[int] = None, patterns: Sequence[Sequence[bool]] = ()):
        """Capture and upload (without running anything) the graphs later replays will use: the
        ``steps``-step group starting at the current step plus the single-step remainders, and/or
        every explicit counting ``pattern`` -- so no capture happens inside a timed region."""
        if steps is not None:
            t = self.step_count
            self._source_graph(tuple(self._counting_at(t + s) for s in range(int(steps))))
            for count in (True, False):
                self._source_graph((count,))
        for p in patterns:
            self._source_graph(tuple(bool(c) for c in p))
        # the source's first permutation too (a 2M-row device randperm costs milliseconds of host
        # time: drawn here, it cannot idle the GPU between a clock settle and the timed steps)
        if hasattr(self._source, "prepare"):
            self._source.prepare(self.step_count, max([1] + [len(p) for p in patterns]))

    def _counting_at(self, t: int) -> bool:
        return self.track_feature_counts and (t % self.count_every == 0)

    def step_source(self, steps: int = 1, pattern: Optional[Sequence[bool]] = None):
        """``steps`` optimizer steps, each on the next batch of the attached source, as ONE graph
        replay (each step: batch gather + the step's kernels; the device step counter indexes the
        batches).  Consecutive graph replays are separated by a ~9 us idle gap on MI355X, so a
        multi-step graph pays it once per ``steps`` steps.  Graphs are captured per pattern of
        feature-counting steps: by default step t counts when ``t % count_every == 0``;
        ``pattern`` (one bool per step) fixes it per replay instead, e.g. count on the first step
        of every group, so one graph serves every group whatever step it starts at."""
        self._tail_ready()
        t = self.step_count
        if pattern is None:
            pattern = tuple(self._counting_at(t + s) for s in range(int(steps)))
        else:
            pattern = tuple(bool(c) and self.track_feature_counts for c in pattern)
            if len(pattern) != int(steps):
                raise ValueError(f"pattern has {len(pattern)} entries for {steps} steps")
        self._source.prepare(t, len(pattern))
        self._source_graph(pattern).replay()
        for count in pattern:
            self._counted = count
            self._host_step()
        return self.out

    def _inputs_graph(self, xs, pattern):
        key = ("inp", tuple(x.data_ptr() for x in xs), tuple(pattern))
        if self._graph is None:
            self._graph = {}
        g = self._graph.get(key)
        if g is None:
            for x in xs:
                if x.dtype != torch.bfloat16 or tuple(x.shape) != (self.batch_size, self.d) or not x.is_contiguous():
                    raise ValueError("graph inputs must be contiguous bf16 [batch_size, d] buffers")
            torch.cuda.synchronize(self.device)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                for x, count in zip(xs, pattern):
                    self._step_kernels(x, count)
            _upload(g, self.device)
            self._graph[key] = g
        return g

    def prime_inputs(self, xs: Sequence[torch.Tensor], pattern: Sequence[bool]):
        """Capture + upload (nothing runs) the multi-step graph ``step_inputs(xs, pattern)`` replays."""
        self._inputs_graph(list(xs), tuple(bool(c) and self.track_feature_counts for c in pattern))

    def step_inputs(self, xs: Sequence[torch.Tensor], pattern: Optional[Sequence[bool]] = None):
        """``len(xs)`` optimizer steps as ONE graph replay, step s on the persistent batch buffer
        ``xs[s]`` (e.g. the all-gathered global batches of a multi-step group under ensemble
        sharding); ``pattern`` = feature counting per step (default: the first step only)."""
        self._tail_ready()
        xs = list(xs)
        if pattern is None:
            pattern = [i == 0 for i in range(len(xs))]
        pattern = tuple(bool(c) and self.track_feature_counts for c in pattern)
        if len(pattern) != len(xs):
            raise ValueError("one counting flag per step")
        self._inputs_graph(xs, pattern).replay()
        for count in pattern:
            self._counted = count
            self._host_step()
        return self.out

    def step_static(self, which: int = 0):
        """Replay the captured step on whatever is in ``x_static`` (fill it first, e.g. with
        ``torch.index_select(..., out=engine.x_static)``), or on static input ``which``."""
        self._tail_ready()
        if self._graph is None:
            self._capture()
        count = self._counting()
        self._counted = count
        self._graph[(count, which)].replay()
        self._host_step()
        return self.out

    @torch.no_grad()
    def evaluate(self, rows: torch.Tensor):
        """FVU and mean L0 of every model on ``rows`` [N, d] (N a multiple of the batch size),
        from the encoder / decoder kernels' own epilogue partials -- no extra passes over the
        codes (reference standard_metrics.py:303-312 computed per model in fp32 torch).
        For centred tied models the FVU is measured in the centred space the model sees.
        Returns (fvu [G], l0 [G]) on the device."""
        B, G = self.batch_size, self.n_models
        N = rows.shape[0] - rows.shape[0] % B
        if N == 0:
            raise ValueError(f"need at least {B} rows")
        se = torch.zeros(G, device=self.device, dtype=torch.float64)
        l0 = torch.zeros(G, device=self.device, dtype=torch.float64)
        s1 = torch.zeros(G, self.d, device=self.device, dtype=torch.float64)
        s2 = torch.zeros(G, device=self.device, dtype=torch.float64)
        for i in range(0, N, B):
            xin = self._x_bf16(rows[i:i + B])
            x = self.prepare(xin)
            gemm_ops.encode_relu(x, self.enc_shadow, self.params[self._bkey], self.c, self.enc_part, None,
                                 self.nactive, mask_out=self.cmask, act=self.act,
                                 ascale=self.s2 if self.kind == "threshold" else None, live_host=self._live)
            if self.kind == "threshold":  # reconstructs the uncentred rows
                x = xin
            gemm_ops.decode_residual(self.c, self.dec_shadow, x, self.r, self.dec_part)
            se += self.dec_part.sum(1).double()
            l0 += self.enc_part[..., 1].sum(1).double()
            xf = x.double() if x.dim() == 3 else x.double().expand(G, B, self.d)
            s1 += xf.sum(1)
            s2 += xf.pow(2).sum((1, 2))
        var = s2 - s1.pow(2).sum(-1) / N  # total sum of squares about the mean
        return (se / var).float(), (l0 / N).float()

    def feature_frequency(self) -> torch.Tensor:
        """Per-feature firing frequency [G, n] = feature_counts / rows_seen.  The counts are SAMPLED:
        the encoder epilogue accumulates them only on counting steps (every ``count_every``-th step, or
        the first step of each multi-step graph replay), and ``rows_seen`` counts exactly those steps'
        rows -- an unbiased estimate of the frequency, not an exact "ever fired" record.  A feature
        that fires only on unsampled steps reads 0 here; consumers that need exact dead-feature
        counts (dead-feature resampling, ``train/huge_batch.py``) build the engine with
        ``count_every=1``."""
        if self.feature_counts is None:
            raise RuntimeError("feature counting is off (track_feature_counts=False)")
        return self.feature_counts / max(1, self.rows_seen)

    def loss_dicts(self, out=None):
        out = (self.out if out is None else out).detach().cpu()
        keys = ["loss", "l_reconstruction", "l_l1", "l_bias_decay", "l0"]
        return [{k: float(out[i, j]) for j, k in enumerate(keys)} for i in range(self.n_models)]

    # ------------------------------------------------------------------ export
    def unstack(self, device="cpu"):
        out = []
        for i in range(self.n_models):
            p = {k: v[i].detach().to(device).clone() for k, v in self.params.items()}
            b = {}
            for k, v in self.models_meta[i].items():
                b[k] = v.detach().to(device).clone() if torch.is_tensor(v) else v
            out.append((p, b))
        return out

    def to_learned_dicts(self, device="cpu"):
        return [self.sig.to_learned_dict(p, b) for p, b in self.unstack(device)]

    def state_dict(self):
        # the bf16 shadows and row norms the kernels read are saved too: rebuilding them from the
        # masters (refresh_shadows) reduces the norms in another order than the Adam kernel that
        # wrote them, so an exact (bit-identical) resume needs the stored ones
        sh = {"enc": self.enc_shadow}
        if self.dec_shadow is not self.enc_shadow:
            sh["dec"] = self.dec_shadow
        return {"kind": self.kind, "params": self.params, "m": self.m, "v": self.v, "lr": self.lr,
                "l1": self.l1, "bias_decay": self.bias_decay, "step": self.step_count,
                "nactive": self.nactive, "feature_counts": self.feature_counts, "rows_seen": self.rows_seen,
                "shadows": sh, "norms": self.norms, "bsq": self._bsq if not self._bsq_dirty else None}

    def load_state_dict(self, sd):
        for k in self.params:
            self.params[k].copy_(sd["params"][k])
            self.m[k].copy_(sd["m"][k])
            self.v[k].copy_(sd["v"][k])
        self.lr.copy_(sd["lr"]); self.l1.copy_(sd["l1"]); self.bias_decay.copy_(sd["bias_decay"])
        self.step_count = int(sd["step"])
        self.step_dev.fill_(self.step_count)
        if sd.get("feature_counts") is not None and self.feature_counts is not None:
            self.feature_counts.copy_(sd["feature_counts"])
        self.rows_seen = int(sd.get("rows_seen", 0))
        sh = sd.get("shadows")
        if sh is not None and sd.get("norms") is not None:
            self.enc_shadow.copy_(sh["enc"])
            if "dec" in sh and self.dec_shadow is not self.enc_shadow:
                self.dec_shadow.copy_(sh["dec"])
            self.norms.copy_(sd["norms"])
            self._bsq_dirty = True
            if sd.get("bsq") is not None and self._bsq is not None:
                self._bsq.copy_(sd["bsq"])  # the fused tail's |b|^2 partials, as the kernel summed them
                self._bsq_dirty = False
        else:  # (older checkpoints: rebuilt from the masters)
            self.refresh_shadows()
