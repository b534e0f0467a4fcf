"""``FusedTopKEnsemble``: top-k dictionary learning for many k in one pass (MI355X path).

Per step, for all models at once (reference runs a Python loop over models because
k differs, ``autoencoders/ensemble.py:100-116``; math of ``autoencoders/topk_encoder.py:19-40``):

1. scores = x D_hat^T                     grouped MFMA GEMM, bf16 epilogue (fp32 accumulation)
2. (idx, val) = top-k(scores), ReLU       per-model k on device; the picks are the fp32 top-k:
                                           bf16 rounding is monotone, so only keys equal to the
                                           k-th largest bf16 key are ambiguous, and those are
                                           ranked by exact fp32 recomputes <x, D_hat[j]>
                                           (``scores_dtype='fp32'``: the fp32 score matrix and
                                           its select; a select fused into the scores GEMM --
                                           candidate append above a sampled bound -- measured
                                           1.51 vs 1.01 ms/step, profiles/r5/topk_candidates/)
3. x_hat = sum val D_hat[idx]; R = x_hat - x; code gradients <R, D_hat[idx]>
                                           one wave per row (sparse gather from L2); the
                                           previous step's dense-buffer picks are cleared here
4. dD_hat = code^T R + dscore^T x          models with small k: feature-major slot lists built
                                           on the device (counting sort) and one wave per
                                           dictionary row summing its picks; the others: ONE
                                           MFMA GEMM with two K segments over the scattered
                                           (dense bf16) code / dscore
5. the step tail, ONE launch (csrc/adam.hip ``sc_topk_tail``): Adam with the row-norm Jacobian
   (D_hat = dict / |dict|) + bf16 shadow, the per-model MSE from the decode's per-row squared errors,
   the next step's batch gather (multi-step source graphs) and the device step counter

``enable_graph()`` captures the whole step as one HIP graph (two, alternating the pick buffers:
step t clears step t-1's picks).
"""

from __future__ import annotations

import os
from typing import Optional, Union

import torch

from ..ops import adam as adam_ops
from ..ops import gemm as gemm_ops
from ..ops import topk as topk_ops

# Cost model of the weight gradient per model (MI355X, measured on config 4): the slot-list
# kernel moves ~4 d bytes per pick at ~5 TB/s from L2 / MALL; the dense two-segment GEMM does
# 4 B n d FLOPs at ~0.9 PF.  A model takes the sparse path when that is clearly cheaper.
_SPARSE_BW = 5.0e12
_DENSE_FLOPS = 0.9e15


def auto_sparse_k(B: int, n: int, d: int, margin: float = 1.3) -> int:
    """Largest k whose slot-list weight gradient beats the dense GEMM by ``margin``."""
    dense = 4.0 * B * n * d / _DENSE_FLOPS
    per_k = B * 4.0 * d / _SPARSE_BW
    return int(dense / (per_k * margin))


class FusedTopKEnsemble:
    def __init__(self, models, sig=None, lr=1e-3, batch_size=256, device="cuda", betas=(0.9, 0.999), eps=1e-8,
                 grad_dtype: str = "bf16", sparse_k: Union[int, str] = "auto", scores_dtype: Optional[str] = None):
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
        ks = [int(m[1]["sparsity"]) for m in models]
        self.k = torch.tensor(ks, dtype=torch.int32, device=dev)
        self.kmax = kmax = max(ks)
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
        # score matrix: bf16 by default (half the HBM round trip of fp32; SC_TOPK_SCORES=fp32 to compare)
        sdt = scores_dtype or os.environ.get("SC_TOPK_SCORES", "bf16")
        if sdt not in ("fp32", "bf16"):
            raise ValueError(f"scores_dtype must be 'fp32' or 'bf16', got {sdt!r}")
        # (a hipBLASLt scores GEMM over the stacked dictionaries with a [B, G, n] select measured no
        # consistent gain over four boxes: scripts/lab/topk_blas_gemmk_r5.patch)
        self.scores = torch.empty(G, B, n, device=dev, dtype=torch.bfloat16 if sdt == "bf16" else torch.float32)
        # pick buffers, alternating per step: the decode of step t zeroes step t-1's picks in the
        # dense code / dscore buffers (no separate clear launch)
        self.idx_buf = torch.zeros(2, G, B, kmax, device=dev, dtype=torch.int32)
        self.val = torch.zeros(G, B, kmax, device=dev)
        self._cur = 0
        self.idx = self.idx_buf[0]
        self.r = torch.empty(G, B, d, device=dev, dtype=bf)
        self.row_se = torch.empty(G, B, device=dev)
        self.codebuf = torch.zeros(G, B, n, device=dev, dtype=bf)
        self.dscbuf = torch.zeros(G, B, n, device=dev, dtype=bf)
        # weight gradient: the leading models with k <= sparse_k from slot lists, the rest dense
        if sparse_k == "auto":
            sparse_k = auto_sparse_k(B, n, d)
        gs = 0
        while gs < G and ks[gs] <= int(sparse_k) and d <= 1024:
            gs += 1
        self.sparse_g = gs
        # the decode scatters codes / code gradients only for the dense-wgrad models (config 4:
        # 1.054 vs 1.059 ms/step scattering for all, profiles/r4/topk_scatter/)
        self._dense_from = gs
        # (decoding the large-k models as dense MFMA GEMMs over the scattered codes measured +3-5 %:
        # scripts/lab/topk_blas_gemmk_r5.patch; every model decodes by the per-row gather)
        self.lists = topk_ops.SlotLists(gs, B, n, ks, kmax, dev) if gs else None
        self.dscv = torch.zeros(G, B, kmax, device=dev) if gs else None
        # bf16 dictionary gradient by default: the dense GEMM's bf16 epilogue + Adam's bf16 loads
        # (config 4: 1.178 -> 1.133 ms/step, profiles/grad_dtype_ab_r2.json); Adam math stays fp32
        if grad_dtype not in ("fp32", "bf16"):
            raise ValueError(f"grad_dtype must be 'fp32' or 'bf16', got {grad_dtype!r}")
        self.g = torch.empty(G, n, d, device=dev, dtype=bf if grad_dtype == "bf16" else torch.float32)
        self.mse = torch.zeros(G, device=dev)
        # fused tail (SC_TOPK_TAIL=0: Adam + torch reductions + counter increment as separate launches)
        self._tail = os.environ.get("SC_TOPK_TAIL", "1") not in ("", "0") and d <= 1024
        self._ticket = torch.zeros(adam_ops.TICKET_INTS, device=dev, dtype=torch.int32)
        self.x_static = torch.zeros(B, d, device=dev, dtype=bf)
        self.use_graph = False
        self._graphs = None
        self._src_graphs = None

    # ------------------------------------------------------------------ the step
    def _step_kernels(self, x, cur: int, gather=None):
        G, B, n, d = self.n_models, self.batch_size, self.n, self.d
        idx, prev = self.idx_buf[cur], self.idx_buf[1 - cur]
        gemm_ops.matmul_nt(x, self.shadow, self.scores)
        topk_ops.topk_select(self.scores, self.k, self.kmax, out=(idx, self.val), x=x, D=self.shadow)
        topk_ops.decode_grad(idx, self.val, self.k, self.shadow, x, self.r, self.row_se, self.codebuf,
                             self.dscbuf, dscv=self.dscv, prev_idx=prev, dense_from=self._dense_from)
        alpha = 2.0 / (B * d)
        gs = self.sparse_g
        if gs:
            topk_ops.slot_lists(idx, self.k, self.lists)
            topk_ops.sparse_wgrad(self.lists, self.val, self.dscv, self.r, x, self.g[:gs], alpha)
        if gs < G:
            gemm_ops.weight_grads([[(self.codebuf[gs:], self.r[gs:]), (self.dscbuf[gs:], x)]], [self.g[gs:]], alpha)
        if self._tail:
            adam_ops.topk_tail(self.params["dict"], self.g, self.m["dict"], self.v["dict"], self.shadow, self.norms,
                               self.lr, *self.betas, self.eps, self.step_dev, self.row_se, self.mse, 1.0 / (B * d),
                               self._ticket, gather=gather)
            return
        torch.mul(torch.sum(self.row_se, dim=1), 1.0 / (B * d), out=self.mse)
        adam_ops.adam_rows([dict(p=self.params["dict"], g=self.g, m=self.m["dict"], v=self.v["dict"],
                                 shadow=self.shadow, norms=self.norms, norm=True)],
                           self.lr, self.step_count + 1, *self.betas, self.eps, step_dev=self.step_dev)
        self.step_dev.add_(1)
        if gather is not None:
            raise RuntimeError("the next-batch gather needs the fused tail")

    def enable_graph(self, enabled: bool = True):
        """Replay the whole step from a HIP graph (one per pick-buffer parity); the batch goes
        through ``x_static``."""
        self.use_graph = enabled
        self._graphs = None
        return self

    def _capture(self):
        torch.cuda.synchronize(self.device)
        self._graphs = []
        for cur in (0, 1):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                self._step_kernels(self.x_static, cur)
            self._graphs.append(g)

    def step_batch(self, batch):
        """One Adam step of every model; returns the per-model MSE (the reference's loss) on device."""
        x = batch if batch is self.x_static else batch.to(self.device, torch.bfloat16).contiguous()
        if self.use_graph:
            if x is not self.x_static:
                self.x_static.copy_(x)
            if self._graphs is None:
                self._capture()
            self._graphs[self._cur].replay()
        else:
            self._step_kernels(x, self._cur)
        self.idx = self.idx_buf[self._cur]
        self._cur ^= 1
        self.step_count += 1
        return self.mse

    def _capture_source(self, source, steps: int, cur0: int):
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            # each step's batch: the first step's own gather kernel; later steps' rows are fetched by the
            # previous step's tail (one launch fewer per step) when the source allows it
            nxt = source.tail_gather(self.x_static) if (self._tail and hasattr(source, "tail_gather")) else None
            for i in range(steps):
                if i == 0 or nxt is None:
                    source.gather(self.x_static, self.step_dev)
                self._step_kernels(self.x_static, cur0 ^ (i & 1), gather=nxt if i + 1 < steps else None)
        return g

    def run_source(self, source, steps: int):
        """``steps`` optimizer steps as ONE graph replay with every batch fetched INSIDE the graph
        (``data.ring.RingGraphSource``: one gather kernel per step on the device step counter), so
        no host sampling or replay boundary sits between steps.  The pick-buffer parity follows the
        step index; graphs are cached per (steps, starting parity)."""
        steps = int(steps)
        if steps < 1:
            raise ValueError("steps must be >= 1")
        if getattr(source, "B", self.batch_size) != self.batch_size:
            raise ValueError("the source's batch size differs from the engine's")
        if self._src_graphs is None or self._src_graphs[0] is not source:
            self._src_graphs = (source, {})
        key = (steps, self._cur)
        graphs = self._src_graphs[1]
        source.prepare(self.step_count, steps)
        if key not in graphs:
            graphs[key] = self._capture_source(source, steps, self._cur)
        graphs[key].replay()
        last = self._cur ^ ((steps - 1) & 1)
        self.idx = self.idx_buf[last]
        self._cur = last ^ 1
        self.step_count += steps
        return self.mse

    # ------------------------------------------------------------------ inference / export
    def encode(self, x):
        """Dense top-k codes [G, B, n] for ``x`` [B, d] with the current dictionaries."""
        xb = x.to(self.device, torch.bfloat16).contiguous()
        # (inference: fp32 scores, so the codes carry the GEMM's fp32 values)
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
