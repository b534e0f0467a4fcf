"""``FusedTopKEnsemble``: top-k dictionary learning for many k in one pass (MI355X path).

Per step, for all models at once (reference runs a Python loop over models because
k differs, ``autoencoders/ensemble.py:100-116``):

1. scores = x D_hat^T                     grouped MFMA GEMM (fp32 out)
2. (idx, val) = top-k(scores), ReLU       radix-select kernel, per-model k on device
3. x_hat = sum val D_hat[idx]; R = x_hat - x; code gradients <R, D_hat[idx]>
                                           one wave per row (sparse gather from L2)
4. dD_hat = code^T R + dscore^T x          ONE MFMA GEMM with two K segments over the
                                           scattered (dense bf16) code / dscore
5. Adam with the row-norm Jacobian (D_hat = dict / |dict|) + bf16 shadow
"""

from __future__ import annotations

import os

import torch

from ..ops import adam as adam_ops
from ..ops import gemm as gemm_ops
from ..ops import topk as topk_ops


class FusedTopKEnsemble:
    def __init__(self, models, sig=None, lr=1e-3, batch_size=256, device="cuda", betas=(0.9, 0.999), eps=1e-8,
                 decode: str = "gather", grad_dtype: str | None = None, score_chunk: int | None = None):
        from ..models.topk import TopKEncoder

        self.sig = sig or TopKEncoder
        self.device = dev = torch.device(device)
        self.n_models = G = len(models)
        self.batch_size = B = int(batch_size)
        self.n, self.d = models[0][0]["dict"].shape
        n, d = self.n, self.d
        if B % 128 or n % 128 or d % 256:
            raise ValueError(f"fused top-k needs B%128==0, n%128==0, d%256==0 (B={B}, n={n}, d={d})")
        self.params = {"dict": torch.stack([m[0]["dict"].detach().float() for m in models]).to(dev).contiguous()}
        self.m = {"dict": torch.zeros_like(self.params["dict"])}
        self.v = {"dict": torch.zeros_like(self.params["dict"])}
        self.k = torch.tensor([int(m[1]["sparsity"]) for m in models], dtype=torch.int32, device=dev)
        self.kmax = int(self.k.max())
        self.meta = [dict(m[1]) for m in models]
        lrs = lr if isinstance(lr, (list, tuple)) else [lr] * G
        self.lr = torch.tensor([float(x) for x in lrs], device=dev)
        self.betas, self.eps = betas, eps
        self.step_count = 0

        self.step_dev = torch.zeros(1, dtype=torch.int32, device=dev)
        bf = torch.bfloat16
        self.shadow = torch.empty(G, n, d, device=dev, dtype=bf)
        self.norms = torch.ones(G, n, device=dev)
        adam_ops.shadow_rows(self.params["dict"], self.shadow, self.norms, normalize=True)
        # Scores GEMM + select in model chunks (``score_chunk`` models at a time, env SC_TOPK_GCHUNK):
        # one chunk's fp32 scores (2 models: 100 MB at config 4) stay resident in the 256 MB MALL
        # between the GEMM that writes them and the select that reads them, instead of a 403 MB
        # round trip through HBM.
        gc = int(score_chunk if score_chunk is not None else os.environ.get("SC_TOPK_GCHUNK", "0") or 0)
        self.g_chunk = G if gc <= 0 else min(G, gc)
        self.scores = torch.empty(self.g_chunk, B, n, device=dev)
        if self.g_chunk < G:
            self._idx_buf = torch.empty(G, B, self.kmax, device=dev, dtype=torch.int32)
            self._val_buf = torch.empty(G, B, self.kmax, device=dev)
        self.r = torch.empty(G, B, d, device=dev, dtype=bf)
        self.row_se = torch.empty(G, B, device=dev)
        self.codebuf = torch.zeros(G, B, n, device=dev, dtype=bf)
        self.dscbuf = torch.zeros(G, B, n, device=dev, dtype=bf)
        # optional split-K weight gradient (SC_TOPK_WSPLIT): 256x256 tiles give only
        # G * (n/256) * (d/256) workgroups (576 for config 4: 2.25 waves over 256 CUs); K halves
        # fill the machine and Adam sums the slabs -- A/B'd slower (1.344 / 1.406 ms for 2 / 3
        # slabs vs 1.318 ms): the extra fp32 slab traffic through Adam costs more than the tail
        self.wg_split = int(os.environ.get("SC_TOPK_WSPLIT", "1"))
        self.wg_cfg = int(os.environ["SC_TOPK_WCFG"]) if os.environ.get("SC_TOPK_WCFG") else None
        self.sc_cfg = int(os.environ["SC_TOPK_SCFG"]) if os.environ.get("SC_TOPK_SCFG") else None
        # optional sparse weight gradient for the leading models whose k / n is small
        # (SC_TOPK_SPARSE_K = the largest k routed there): the dense GEMM costs the same for every
        # model, the slot-list form is proportional to k -- but one wave per dictionary row
        # (A/B: profiles/README.md)
        sparse_k = int(os.environ.get("SC_TOPK_SPARSE_K", "0"))
        ks = [int(m[1]["sparsity"]) for m in models]
        gs = 0
        while gs < G and ks[gs] <= sparse_k:
            gs += 1
        self.sparse_g = gs if d % 256 == 0 and d <= 1024 else 0
        self._ks, self._sp_cache = ks, {}
        self.dscv = torch.zeros(G, B, self.kmax, device=dev) if self.sparse_g else None
        # bf16 dictionary gradient (default; ``grad_dtype`` / env SC_GRAD_DTYPE): the weight-gradient
        # GEMM's bf16 epilogue + Adam's bf16-gradient loads (dense GEMM path, no split-K).  Config 4
        # A/B: 1.178 -> 1.133 ms/step (profiles/grad_dtype_ab_r2.json); Adam math stays fp32
        gdt = grad_dtype or os.environ.get("SC_GRAD_DTYPE", "bf16")
        if gdt not in ("fp32", "bf16"):
            raise ValueError(f"grad_dtype must be 'fp32' or 'bf16', got {gdt!r}")
        gbf = gdt == "bf16" and self.wg_split == 1 and not self.sparse_g
        self.g_all = torch.empty(self.wg_split, G, n, d, device=dev, dtype=bf if gbf else torch.float32)
        self.g = self.g_all[0]
        self.idx = self.val = None
        # fold the dense-buffer clear into the next step's decode (SC_TOPK_FOLD_CLEAR, default on)
        self.fold_clear = os.environ.get("SC_TOPK_FOLD_CLEAR", "1") not in ("", "0")
        self._prev_idx = None
        # decode: "gather" (sparse, one wave per row) or "gemm" (dense codes through the decoder and
        # code-gradient epilogue GEMMs); chosen from measurement (profiles/config4_topk_r2.json)
        self.decode = decode
        self.dec_part = torch.zeros(G, (B // 128) * (d // 128), device=dev)
        self._colpart = torch.zeros(G, B // 128, n, device=dev)
        self._zero_l1 = torch.zeros(G, device=dev)
        self._se = torch.zeros(G, device=dev)

    def step_batch(self, batch):
        x = batch.to(self.device, torch.bfloat16).contiguous()
        G, B, n, d = self.n_models, self.batch_size, self.n, self.d
        gc = self.g_chunk
        for g0 in range(0, G, gc):
            g1 = min(G, g0 + gc)
            sc = self.scores[: g1 - g0]
            if self.sc_cfg is not None:  # A/B knob SC_TOPK_SCFG: block shape of the scores GEMM
                with gemm_ops.force_shape(self.sc_cfg):
                    gemm_ops.matmul_nt(x, self.shadow[g0:g1], sc)
            else:
                gemm_ops.matmul_nt(x, self.shadow[g0:g1], sc)
            if gc >= G:
                self.idx, self.val = topk_ops.topk_select(sc, self.k, self.kmax)
            else:
                topk_ops.topk_select(sc, self.k[g0:g1], self.kmax, out=(self._idx_buf[g0:g1], self._val_buf[g0:g1]))
                self.idx, self.val = self._idx_buf, self._val_buf
        if self.decode == "gemm":
            # dense-GEMM decode: scatter the codes, R = codes D_hat - x (decoder-epilogue GEMM,
            # sum R^2 partials), code gradients 1[c > 0] (R D_hat^T) (code-gradient epilogue GEMM)
            topk_ops.scatter(self.idx, self.val, self.k, self.codebuf)
            gemm_ops.decode_residual(self.codebuf, self.shadow, x, self.r, self.dec_part)
            gemm_ops.code_grad(self.r, self.shadow, self.codebuf, self._zero_l1, self.dscbuf, self._colpart)
            torch.sum(self.dec_part, dim=1, out=self._se)
        else:
            # gather decode: one wave per row, k dictionary rows gathered twice from L2 / MALL
            topk_ops.decode_grad(self.idx, self.val, self.k, self.shadow, x, self.r, self.row_se, self.codebuf,
                                 self.dscbuf, dscv=self.dscv, prev_idx=self._prev_idx if self.fold_clear else None)
            torch.sum(self.row_se, dim=1, out=self._se)
        gs = self.sparse_g if self.decode == "gather" else 0
        if gs:
            topk_ops.sparse_wgrad(self.idx, self.val, self.dscv, self._ks, self.r, x, self.g[:gs], 2.0 / (B * d),
                                  cache=self._sp_cache)
        if gs == G:
            pass
        elif gs:
            gemm_ops.weight_grads([[(self.codebuf[gs:], self.r[gs:]), (self.dscbuf[gs:], x)]], [self.g[gs:]],
                                  2.0 / (B * d))
        elif self.wg_split > 1:
            gemm_ops.weight_grads([[(self.codebuf, self.r), (self.dscbuf, x)]], [self.g_all], 2.0 / (B * d),
                                  ksplit=self.wg_split)
        elif self.wg_cfg is not None:  # A/B knob SC_TOPK_WCFG: block shape of the weight gradient
            with gemm_ops.force_shape(self.wg_cfg):
                gemm_ops.weight_grads([[(self.codebuf, self.r), (self.dscbuf, x)]], [self.g], 2.0 / (B * d))
        else:
            gemm_ops.weight_grads([[(self.codebuf, self.r), (self.dscbuf, x)]], [self.g], 2.0 / (B * d))
        if self.fold_clear and self.decode == "gather":
            # the next step's decode zeroes these picks (one launch less per step); the idx tensor
            # must survive until then (in the one-shot path topk_select returns a fresh one per step)
            self._prev_idx = self.idx.clone() if self.g_chunk < G else self.idx
        else:
            topk_ops.clear(self.idx, self.codebuf, self.dscbuf)
        adam_ops.adam_rows([dict(p=self.params["dict"], g=self.g, m=self.m["dict"], v=self.v["dict"],
                                 shadow=self.shadow, norms=self.norms, norm=True)],
                           self.lr, self.step_count + 1, *self.betas, self.eps, step_dev=self.step_dev,
                           nsplit=self.wg_split, gstride=G * n * d)
        self.step_dev += 1
        self.step_count += 1
        return self._se / (B * d)  # per-model MSE (the reference's loss), on device

    def encode(self, x):
        """Dense top-k codes [G, B, n] for ``x`` [B, d] with the current dictionaries."""
        xb = x.to(self.device, torch.bfloat16).contiguous()
        scores = torch.empty(self.n_models, x.shape[0], self.n, device=self.device)
        gemm_ops.matmul_nt(xb, self.shadow, scores)
        idx, val = topk_ops.topk_select(scores, self.k, self.kmax)
        # slots >= k[g] are padded with (index 0, value 0): scatter_add keeps a real pick of
        # feature 0 intact (real indices are unique, the padded values add 0)
        return torch.zeros_like(scores).scatter_add_(-1, idx.long(), val)

    def unstack(self, device="cpu"):
        return [({"dict": self.params["dict"][i].detach().to(device).clone()},
                 {k: (v.detach().to(device).clone() if torch.is_tensor(v) else v) for k, v in self.meta[i].items()})
                for i in range(self.n_models)]

    def to_learned_dicts(self, device="cpu"):
        return [self.sig.to_learned_dict(p, b) for p, b in self.unstack(device)]
