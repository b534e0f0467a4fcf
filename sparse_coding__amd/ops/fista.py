"""FISTA sparse coding for a whole ensemble: the gfx950 persistent kernel
(``csrc/fista.hip``) plus the batched-torch oracle it is tested against.

Reference: ``autoencoders/fista.py:99-128`` (solver) and ``:131-138`` (quadratic
basis update).  Shapes: X [G, B, d] (or [B, d] shared by all models), D [G, n, d]
row-normalised dictionaries, warm start A0 [G, B, n], lam / eta [G].
"""

from __future__ import annotations

import math
from typing import Optional, Tuple

import numpy as np
import torch

from . import _lib


def momentum_schedule(iters: int) -> torch.Tensor:
    """mom[t] = (t_k - 1) / t_{k+1} with t_1 = 1, t_{k+1} = (1 + sqrt(1 + 4 t_k^2)) / 2."""
    mom = np.empty(iters, dtype=np.float64)
    tk_n = 1.0
    for t in range(iters):
        tk = tk_n
        tk_n = (1.0 + math.sqrt(1.0 + 4.0 * tk * tk)) / 2.0
        mom[t] = (tk - 1.0) / tk_n
    return torch.from_numpy(mom.astype(np.float32))


def step_size(D: torch.Tensor, method: str = "eigh", iters: int = 30) -> torch.Tensor:
    """eta = 1 / lambda_max(D D^T) per model (reference uses eigvalsh, :104-106).

    ``method="power"`` runs batched power iteration on D^T D ([d, d], cheaper when
    n > d) with a 1% safety margin so eta never exceeds the true 1/L.
    """
    D = D.float()
    if method == "eigh":
        gram = D @ D.transpose(-1, -2)
        return 1.0 / torch.linalg.eigvalsh(gram).amax(dim=-1)
    G, n, d = D.shape
    gram = D.transpose(-1, -2) @ D  # same nonzero spectrum, [d, d]
    v = torch.randn(G, d, 1, device=D.device, generator=torch.Generator(D.device).manual_seed(0))
    for _ in range(iters):
        v = gram @ v
        v = v / v.norm(dim=1, keepdim=True)
    lam_max = (v.transpose(1, 2) @ gram @ v).squeeze(-1).squeeze(-1)
    return 1.0 / (1.01 * lam_max)


class EtaTracker:
    """eta = 1 / lambda_max(D D^T) for a dictionary that changes a little every step.

    The reference recomputes the full spectrum (``eigvalsh`` of [n, n], rocSOLVER:
    ~3 ms per model at n = 1024) on every FISTA call.  Between steps the basis update
    moves D by ~1e-3, so the top eigenvector barely moves: warm-started power iteration
    from the previous eigenvector (``warm_iters`` products with D^T D, [d, d]) gives the
    Rayleigh quotient to O(angle^2), and an exact ``eigh`` refresh every
    ``refresh_every`` calls bounds drift.  ``margin`` keeps eta on the safe side of 1/L
    (the quotient approaches lambda_max from below).
    """

    def __init__(self, refresh_every: int = 50, warm_iters: int = 4, margin: float = 1e-3):
        self.refresh_every = refresh_every
        self.warm_iters = warm_iters
        self.margin = margin
        self.v = None
        self.calls = 0
        self.space = "dtd"  # which Gram the eigenvector lives in: D^T D [d, d] or D D^T [n, n]

    def __call__(self, D: torch.Tensor) -> torch.Tensor:
        D = D.float()
        return self._track(D.transpose(-1, -2) @ D, "dtd")  # [G, d, d], same nonzero spectrum as D D^T

    def from_gram(self, gram: torch.Tensor) -> torch.Tensor:
        """The same estimate from a Gram matrix D D^T [G, n, n] fp32 the caller already has -- the
        solver's own (``gram_solve``: bf16 D, fp32 accumulation), so eta bounds the operator the
        iterations actually apply and no separate fp32 D^T D product is needed."""
        return self._track(gram, "ddt")

    def _track(self, gram: torch.Tensor, space: str) -> torch.Tensor:
        if space != self.space:  # the warm eigenvector belongs to the other Gram: refresh exactly
            self.space, self.v = space, None
        if self.v is None or self.v.shape[:2] != gram.shape[:2] or self.calls % self.refresh_every == 0:
            vals, vecs = torch.linalg.eigh(gram)
            self.v = vecs[..., -1:].contiguous()
            self.calls += 1
            return 1.0 / vals[..., -1]
        v = self.v
        for _ in range(self.warm_iters):
            v = gram @ v
            v = v / v.norm(dim=1, keepdim=True)
        self.v = v
        self.calls += 1
        lam = (v.transpose(1, 2) @ gram @ v).reshape(-1)
        return 1.0 / ((1.0 + self.margin) * lam)

    def state_dict(self):
        return {"v": None if self.v is None else self.v.detach().clone(), "calls": self.calls, "space": self.space}

    def load_state_dict(self, st):
        self.v = None if st.get("v") is None else st["v"].clone()
        self.calls = int(st.get("calls", 0))
        self.space = st.get("space", "dtd")


def fista_torch(X, D, lam, A0=None, iters=500, eta=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Batched fp32 oracle: identical arithmetic to the reference loop, all models at once."""
    D = D.float()
    G, n, d = D.shape
    X = X.float()
    if X.dim() == 2:
        X = X.expand(G, *X.shape)
    if eta is None:
        eta = step_size(D)
    eta = eta.to(D.device).float().view(G, 1, 1)
    lam = torch.as_tensor(lam, device=D.device, dtype=torch.float32).view(G, 1, 1)
    A = torch.zeros(G, X.shape[1], n, device=D.device) if A0 is None else A0.float().clone()
    Y = A.clone()
    mom = momentum_schedule(iters).tolist()
    Dt = D.transpose(1, 2)
    for t in range(iters):
        A_prev = A
        res = X - torch.bmm(Y, D)
        Y = Y + eta * torch.bmm(res, Dt)
        A = torch.clamp(Y - eta * lam, min=0.0)
        Y = A + (A - A_prev) * mom[t]
    return A, X - torch.bmm(A, D)


GRAM_N = (256, 512, 768, 1024)
# (d / 128, n / 128) instantiated for the direct-form solver (csrc/fista.hip sc_fista)
DIRECT_TILES = {(2, 2), (2, 4), (2, 8), (2, 16), (4, 4), (4, 8), (4, 16), (6, 6), (6, 12), (8, 4), (8, 8), (8, 16)}


def fista(X, D, lam, A0=None, iters=500, eta=None, backend: str = "auto", with_res: bool = True,
          form: str = "auto", rows: int = 0) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """Solve min_A>=0 1/2|X - A D|^2 + lam |A|_1 (ISTA step eta) for every model.

    backend: "hip" (gfx950 kernel, bf16 GEMM operands, fp32 iterates), "torch" (fp32
    oracle), or "auto" (hip when the GPU kernel supports the shape).
    form (hip only): "direct" -- two products per iteration, (Y D) then (Res D^T);
    "gram" -- Y += eta (X D^T - Y (D D^T)), one [B, n] x [n, n] product per iteration
    (2 B n^2 instead of 4 B n d FLOPs); "auto" picks gram for n <= d.
    rows (hip only): batch rows per workgroup, 16 or 32 where that form is instantiated; 0 lets
    the kernel library choose (32 when that still gives enough workgroups to fill the chip).
    """
    if rows not in (0, 16, 32):
        raise ValueError(f"rows must be 0, 16 or 32, got {rows}")
    G, n, d = D.shape
    B = X.shape[-2]
    use_hip = backend == "hip" or (backend == "auto" and D.is_cuda and _lib.available() and B % 16 == 0
                                   and n % 128 == 0 and d % 128 == 0)
    if not use_hip:
        return fista_torch(X, D, lam, A0, iters, eta)
    dev = D.device
    if eta is None:
        eta = step_size(D)
    eta = eta.to(dev).float().contiguous()
    lam = torch.as_tensor(lam, device=dev, dtype=torch.float32).reshape(G).contiguous()
    Xb = X.to(torch.bfloat16).contiguous()  # [B, d] stays shared: the grouped GEMMs take a stride-0 operand
    Db = D.to(torch.bfloat16).contiguous()
    A = torch.empty(G, B, n, device=dev)
    a0 = _f32(A0) if A0 is not None else None
    mom = momentum_schedule(max(iters, 1)).to(dev)
    if form == "auto":
        form = "gram" if (n <= d and n in GRAM_N) else "direct"
    if form == "gram" and n in GRAM_N and B % 16 == 0:
        from . import gemm

        C = torch.empty(G, B, n, device=dev)
        if B % 128 == 0:
            gemm.matmul_nt(Xb, Db, C)                   # C = X D^T (MFMA, fp32 out)
        else:
            torch.matmul(Xb.float(), Db.float().transpose(1, 2), out=C)
        Gm = torch.empty(G, n, n, device=dev, dtype=torch.bfloat16)
        gemm.matmul_nt(Db, Db, Gm)                      # Gm = D D^T (bf16 out)
        # MFMA-fragment order (constant over the solve): [G][n/16 col tiles][n/32 k-steps][q][row][8]
        # so every wave fragment load is 1 KB contiguous (8 full lines instead of 16 half lines)
        Gm = Gm.view(G, n // 16, 16, n // 32, 4, 8).permute(0, 1, 3, 4, 2, 5).contiguous()
        rc = _lib.lib().sc_fista_gram(_lib.ptr(C), _lib.ptr(Gm), _lib.ptr(a0), _lib.ptr(eta), _lib.ptr(lam),
                                      _lib.ptr(mom), _lib.ptr(A), G, B, n, iters, _lib.stream_handle(), rows, 0,
                                      None, None, None, None, None)
    else:
        if Xb.dim() == 2:  # (the direct-form solver reads a per-model X)
            Xb = Xb.expand(G, *Xb.shape).contiguous()
        # both operands in MFMA-fragment order (see the Gram form): D [G][n/16][d/32][64][8] for the
        # (Res D^T) product, D^T [G][d/16][n/32][64][8] for the (Y D) product
        Dtb = Db.transpose(1, 2).reshape(G, d // 16, 16, n // 32, 4, 8).permute(0, 1, 3, 4, 2, 5).contiguous()
        Dfb = Db.view(G, n // 16, 16, d // 32, 4, 8).permute(0, 1, 3, 4, 2, 5).contiguous()
        rc = _lib.lib().sc_fista(_lib.ptr(Xb), _lib.ptr(Dfb), _lib.ptr(Dtb), _lib.ptr(a0), _lib.ptr(eta),
                                 _lib.ptr(lam), _lib.ptr(mom), _lib.ptr(A), 0, G, B, n, d, iters, None, None, None,
                                 _lib.stream_handle(), rows)
    if rc == 2 and backend == "auto":
        return fista_torch(X, D, lam, A0, iters, eta)
    _lib.check(rc, "sc_fista")
    if not with_res:
        return A, None
    # final residual in fp32 against the exact dictionary (one plain GEMM per model)
    Xf = X.float() if X.dim() == 3 else X.float().expand(G, *X.shape)
    return A, Xf - torch.bmm(A, D.float())


def _f32(t: torch.Tensor) -> torch.Tensor:
    """``t`` as contiguous fp32 without a copy when it already is."""
    return t if (t.dtype == torch.float32 and t.is_contiguous()) else t.float().contiguous()


def gram_fragments(gm32: torch.Tensor) -> torch.Tensor:
    """fp32 Gram [G, n, n] -> the Gram solver's bf16 MFMA-fragment order
    [G][n/16 col tiles][n/32 k-steps][q][row][8] in one cast + permute pass."""
    G, n, _ = gm32.shape
    out = torch.empty(G, n // 16, n // 32, 4, 16, 8, device=gm32.device, dtype=torch.bfloat16)
    out.copy_(gm32.view(G, n // 16, 16, n // 32, 4, 8).permute(0, 1, 3, 4, 2, 5))
    return out


def gram_solve_ok(X, D) -> bool:
    """Shapes the dictionary-update hot path (``gram_solve``) takes: the Gram-form solver and the
    step GEMMs (B, d multiples of 128, n one of GRAM_N and n <= d)."""
    G, n, d = D.shape
    return (D.is_cuda and _lib.available() and X.shape[-2] % 128 == 0 and d % 128 == 0 and n in GRAM_N
            and n <= d and X.dim() == 2)


def gram_solve(X, D, lam, A0, iters, eta=None, tracker: Optional[EtaTracker] = None, rows: int = 0):
    """The GPU hot path of one FISTA dictionary step (``models.fista.FistaDictUpdater``): everything the
    basis update needs, with no fp32 GEMM and no operand copies.

    * C = X D^T and Gm = D D^T on the MFMA GEMM (bf16 operands, fp32 out; X [B, d] shared by the models);
    * eta from ``tracker.from_gram(Gm)`` (the Gram the iterations apply) unless given;
    * the persistent Gram-form solve (A fp32);
    * Ab = bf16(A) once, and the NEGATED residual Rn = A D - X (bf16) by the decoder GEMM's EPI_DEC
      epilogue, with per-tile sum(R^2) partials -- replacing the fp32 ``torch.bmm`` residual of
      ``fista()`` (the basis update rounds A and the residual to bf16 for its own GEMM anyway).

    Returns (A fp32 [G, B, n], Ab bf16, Rn bf16 [G, B, d], eta [G], se [G] = |X - A D|^2 per model).
    Reference: ``autoencoders/fista.py:99-128`` (solve) and ``:131-138`` (the residual it hands on)."""
    from . import gemm

    G, n, d = D.shape
    B = X.shape[-2]
    dev = D.device
    Xb = X.to(torch.bfloat16).contiguous()
    Db = D.to(torch.bfloat16).contiguous()
    C = torch.empty(G, B, n, device=dev)
    gemm.matmul_nt(Xb, Db, C)
    gm32 = torch.empty(G, n, n, device=dev)
    gemm.matmul_nt(Db, Db, gm32)
    if eta is None:
        eta = tracker.from_gram(gm32) if tracker is not None else 1.0 / torch.linalg.eigvalsh(gm32).amax(dim=-1)
    eta = eta.to(dev).float().contiguous()
    Gm = gram_fragments(gm32)
    del gm32
    lam = torch.as_tensor(lam, device=dev, dtype=torch.float32).reshape(G).contiguous()
    A = torch.empty(G, B, n, device=dev)
    mom = momentum_schedule(max(iters, 1)).to(dev)
    rc = _lib.lib().sc_fista_gram(_lib.ptr(C), _lib.ptr(Gm), _lib.ptr(_f32(A0) if A0 is not None else None),
                                  _lib.ptr(eta), _lib.ptr(lam), _lib.ptr(mom), _lib.ptr(A), G, B, n, iters,
                                  _lib.stream_handle(), rows, 0, None, None, None, None, None)
    _lib.check(rc, "sc_fista_gram")
    Ab = A.to(torch.bfloat16)
    Rn = torch.empty(G, B, d, device=dev, dtype=torch.bfloat16)
    part = torch.empty(G, (B // 128) * (d // 128), device=dev)
    gemm.decode_residual(Ab, Db, Xb, Rn, part)
    return A, Ab, Rn, eta, part.sum(dim=1)


def _hip_ok(*ts) -> bool:
    return all(t.is_cuda for t in ts) and _lib.available()


def hessian_ema(H, A, history: int = 300, backend: str = "auto"):
    """H <- H (history-1)/history + mean_b(A^2)/history (reference fista.py:91-92).

    HIP path (``backend`` "hip" / "auto" on the GPU): one column-reduction kernel for every
    model (csrc/fista_update.hip); returns a new tensor either way."""
    G, B, n = A.shape
    if backend == "torch" or not (_hip_ok(A, H) and n % 64 == 0):
        return H * ((history - 1.0) / history) + A.pow(2).mean(dim=-2) / history
    out = H.float().contiguous().clone()
    rc = _lib.lib().sc_hessian_ema(_lib.ptr(A.float().contiguous()), _lib.ptr(out), G, B, n, float(history),
                                   _lib.stream_handle())
    _lib.check(rc, "sc_hessian_ema")
    return out


def quadratic_basis_update(D, Res, A, H, lowest_activation=0.001, step=0.001, nonneg=False,
                           normalize: str = "column", backend: str = "auto", shadow_out=None,
                           A_bf16=None, res_neg_bf16=None):
    """D' = D + (step Res^T A / B / (H + lowest))^T, then renormalise (reference :131-138).

    normalize="column" reproduces the reference (``D.norm(2, 0)``: per activation
    dimension, SURVEY B#4); "row" normalises each atom (the intended unit-norm dictionary).
    Batched over models: D [G, n, d], Res [G, B, d], A [G, B, n], H [G, n].

    HIP path: A^T Res by the grouped MFMA GEMM (bf16 operands, fp32 accumulation, the
    step/B scale in its epilogue), then one kernel adds the H-scaled update, clamps and
    renormalises (csrc/fista_update.hip); ``shadow_out`` (bf16 [G, n, d]) optionally receives
    the bf16 copy the next solve multiplies by.  ``A_bf16`` / ``res_neg_bf16`` (HIP path, from
    ``gram_solve``): the GEMM operands already in bf16, the residual NEGATED (A D - X); ``Res`` may
    then be None.
    """
    G, B, n = A.shape
    d = D.shape[-1]
    if Res is None and res_neg_bf16 is None:
        raise ValueError("quadratic_basis_update needs Res or res_neg_bf16")
    hip = (backend != "torch" and _hip_ok(D, A, H) and (Res is None or Res.is_cuda) and n % 128 == 0
           and d % 128 == 0 and B % 64 == 0)
    if not hip and Res is None:
        Res = -res_neg_bf16.float()
    if not hip:
        dB = step * torch.bmm(Res.transpose(1, 2).float(), A.float()) / B  # [G, d, n]
        dB = dB / (H.unsqueeze(1) + lowest_activation)
        D = D.float() + dB.transpose(1, 2)
        if nonneg:
            D = D.clamp(min=0.0)
        out = D / D.norm(dim=1, keepdim=True) if normalize == "column" else D / D.norm(dim=2, keepdim=True).clamp(min=1e-8)
        if shadow_out is not None:
            shadow_out.copy_(out)
        return out
    from . import gemm

    dBt = torch.empty(G, n, d, device=D.device)
    if res_neg_bf16 is not None:  # A^T (A D - X) = -A^T Res
        Ab = A_bf16 if A_bf16 is not None else A.to(torch.bfloat16)
        gemm.weight_grads([[(Ab.contiguous(), res_neg_bf16.contiguous())]], [dBt], -step / B)
    else:
        gemm.weight_grads([[(A.to(torch.bfloat16).contiguous(), Res.to(torch.bfloat16).contiguous())]], [dBt], step / B)
    out = D.float().contiguous().clone()
    rc = _lib.lib().sc_basis_apply(_lib.ptr(out), _lib.ptr(dBt), _lib.ptr(_f32(H)),
                                   _lib.ptr(shadow_out), G, n, d, float(lowest_activation), int(bool(nonneg)),
                                   1 if normalize == "row" else 0, _lib.stream_handle())
    _lib.check(rc, "sc_basis_apply")
    return out


# --------------------------------------------------------------------- FISTA in the loss
class _TrackedEta(torch.autograd.Function):
    """eta = 1 / lambda_max(D D^T) from an ``EtaTracker`` (warm power iteration), differentiable
    in D: with u the top right singular vector of D (the tracker's eigenvector of D^T D),
    d lambda_max / dD = 2 (D u) u^T, so dD = etabar * (-eta^2) * 2 (D u) u^T."""

    @staticmethod
    def forward(ctx, D, tracker):
        eta = tracker(D.detach())
        u = tracker.v.detach().to(D.dtype)  # [G, d, 1]
        ctx.save_for_backward(D.detach(), u, eta)
        return eta

    @staticmethod
    def backward(ctx, etabar):
        D, u, eta = ctx.saved_tensors
        Du = torch.bmm(D, u)                                          # [G, n, 1]
        scale = (-2.0 * etabar * eta * eta).to(D.dtype)[:, None, None]
        return scale * torch.bmm(Du, u.transpose(1, 2)), None


def tracked_eta(D, tracker: "EtaTracker"):
    """Differentiable eta for the FISTA-in-the-loss objective (reference fista.py:104-106 computes
    it from the differentiable normalised encoder and does not detach it)."""
    return _TrackedEta.apply(D, tracker)


def exact_eta(D):
    """eta = 1 / eigvalsh(D D^T).max() per model, differentiable (torch's eigvalsh backward)."""
    return 1.0 / torch.linalg.eigvalsh(D @ D.transpose(-1, -2)).amax(dim=-1)


def unrolled_fista_plain(X, D, lam, A0, iters: int, eta):
    """The unrolled iterations as plain differentiable torch ops (reference fista.py:141-172
    verbatim semantics): used under functorch transforms (vmap / grad of a signature loss),
    where the explicit-adjoint autograd Function does not apply.  D [G, n, d], X [B, d] or
    [G, B, d], A0 [G, B, n], lam / eta [G]."""
    G = D.shape[0]
    e = torch.as_tensor(eta, dtype=D.dtype, device=D.device).reshape(-1)
    e = e.expand(G)[:, None, None] if e.numel() == 1 else e[:, None, None]
    lam = torch.as_tensor(lam, dtype=D.dtype, device=D.device).reshape(-1)
    thr = e * (lam.expand(G)[:, None, None] if lam.numel() == 1 else lam[:, None, None])
    Dt = D.transpose(1, 2)
    mom = momentum_schedule(max(iters, 1)).tolist()
    A = A0
    Y = A0
    for t in range(iters):
        A_prev = A
        res = X - Y @ D
        A = torch.relu(Y + e * (res @ Dt) - thr)
        Y = A + (A - A_prev) * mom[t]
    return X - A @ D


def unrolled_fista_residual(X, D, lam, A0, iters: int = 50, eta=None, backend: str = "auto"):
    """R = X - A_T D after ``iters`` unrolled FISTA iterations warm-started at A0, differentiable
    in D, A0 and eta -- the "FISTA in the loss" term of reference autoencoders/fista.py:141-172
    for every model at once (D [G, n, d], X [B, d] or [G, B, d], A0 [G, B, n], lam / eta [G]).
    ``eta=None`` computes 1 / lambda_max(D D^T) differentiably, as the reference does (its
    eigvalsh is not detached); a given ``eta`` tensor that requires grad receives
    dL/deta = sum_t <Vbar_t, Res_t D^T - lam> from the adjoint sweep.

    Forward: the direct-form HIP solver saving the bf16 iterate slabs Y_t, Res_t, A_{t+1}
    ([G][T][B][*], 288 GB of HBM makes storing every iterate the cheap option).  Backward: the
    adjoint sweep t = T-1 .. 0, per iteration two grouped MFMA GEMMs (nS = -(Vbar D),
    nS D^T) and one elementwise kernel; the dictionary gradient of all T iterations is ONE
    K-concatenated GEMM over the slabs:  Dbar = eta sum_t (Vbar_t^T Res_t - Y_t^T S_t)
    - A_T^T Rbar.  ``backend="torch"`` runs the same adjoint in fp32 torch (the CPU path)."""
    D = D if D.dim() == 3 else D[None]
    G = D.shape[0]
    lam = torch.as_tensor(lam, dtype=torch.float32, device=D.device).reshape(-1).expand(G).contiguous()
    if eta is None:
        eta = exact_eta(D.float())
    eta = torch.as_tensor(eta, dtype=torch.float32, device=D.device).reshape(-1).expand(G).contiguous()
    return _UnrolledFista.apply(X, D, A0, lam, eta, int(iters), backend)


def _unrolled_hip_ok(X, D, A0, backend):
    if backend == "torch":
        return False
    G, n, d = D.shape
    B = A0.shape[-2]
    ok = (_hip_ok(D) and B % 128 == 0 and n % 128 == 0 and d % 128 == 0
          and ((d // 128, n // 128) in DIRECT_TILES or _gram_unrolled_ok(D, A0)))
    if backend == "hip" and not ok:
        raise ValueError(f"unrolled FISTA HIP path needs B % 128 == 0 and (d/128, n/128) in {sorted(DIRECT_TILES)} "
                         f"or the Gram form (n in {GRAM_N}, n <= d, d % 256 == 0) (B={B}, n={n}, d={d})")
    return ok


class _UnrolledFista(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, D, A0, lam, eta, iters, backend):
        G, n, d = D.shape
        B = A0.shape[-2]
        mom = momentum_schedule(max(iters, 1))
        ctx.iters, ctx.mom = iters, mom.tolist()
        ctx.x_shape = X.shape
        if _unrolled_hip_ok(X, D, A0, backend):
            ctx.gram = _gram_unrolled_ok(D, A0) and iters >= 1
            if ctx.gram:
                R, st = unrolled_forward_gram(X.detach(), D.detach(), A0.detach(), lam, eta.detach(), iters, mom)
                ctx.hip = True
                ctx.save_for_backward(*st, eta.detach(), lam)
                return R
            R, Db, Ys, Rs, As = unrolled_forward_hip(X, D.detach(), A0.detach(), lam, eta, iters, mom)
            ctx.hip = True
            ctx.save_for_backward(Db, Ys, Rs, As, eta.detach(), lam)
            return R
        ctx.hip = False
        Df = D.detach().float()
        Xf = X.detach().float()
        e = eta.detach()[:, None, None]
        thr = (eta.detach() * lam)[:, None, None]
        A = A0.detach().float()
        Y = A
        Ys, Rs, As = [], [], []
        for t in range(iters):
            Res = Xf - Y @ Df
            Ys.append(Y)
            Rs.append(Res)
            A_prev = A
            A = torch.clamp(Y + e * (Res @ Df.transpose(1, 2)) - thr, min=0.0)
            As.append(A)
            Y = A + (A - A_prev) * ctx.mom[t]
        R = Xf - A @ Df
        ctx.save_for_backward(Df, torch.stack(Ys, 1) if Ys else None, torch.stack(Rs, 1) if Rs else None,
                              torch.stack(As, 1) if As else None, eta.detach(), A, lam)
        return R

    @staticmethod
    def backward(ctx, Rbar):
        want_eta = ctx.needs_input_grad[4]
        if ctx.hip and ctx.gram:
            *st, eta, lam = ctx.saved_tensors
            Dbar, cbar, etabar = unrolled_backward_gram(Rbar, tuple(st), eta, ctx.mom, ctx.iters,
                                                        lam=lam if want_eta else None)
            return None, Dbar, cbar, None, etabar, None, None
        if ctx.hip:
            Db, Ys, Rs, As, eta, lam = ctx.saved_tensors
            Dbar, cbar, etabar = unrolled_backward_hip(Rbar, Db, Ys, Rs, As, eta, ctx.mom, ctx.iters,
                                                       lam=lam if want_eta else None)
            return None, Dbar, cbar, None, etabar, None, None
        Df, Ys, Rs, As, eta, A_T, lam = ctx.saved_tensors
        Dbar, cbar, etabar = unrolled_backward_torch(Rbar, Df, Ys, Rs, As, eta, ctx.mom, ctx.iters, A_T,
                                                     lam=lam if want_eta else None)
        return None, Dbar, cbar, None, etabar, None, None


def unrolled_backward_torch(Rbar, Df, Ys, Rs, As, eta, mom, T, A_T=None, lam=None):
    """fp32 adjoint sweep over saved iterate slabs ([G][T][B][*], any float dtype): the
    reference arithmetic for ``_unrolled_backward_hip`` (given the same slabs, the two differ
    only by the bf16 rounding of Vbar / S and of the GEMM operands).  Returns (Dbar, cbar,
    etabar); etabar = sum_t <S_t, Res_t> - lam sum Vbar_t (S_t = Vbar_t D: iteration t's
    pre-activation is Y_t + eta (Res_t D^T - lam)) when ``lam`` is given, else None."""
    Df = Df.float()
    e = eta[:, None, None]
    Rbar = Rbar.float()
    Dt = Df.transpose(1, 2)
    if A_T is None:
        A_T = As[:, T - 1]
    Dbar = -A_T.float().transpose(1, 2) @ Rbar
    etabar = torch.zeros_like(eta) if lam is not None else None
    if T == 0:
        return Dbar, -Rbar @ Dt, etabar
    Vbar = -(Rbar @ Dt) * (As[:, T - 1] > 0)
    Ynext = torch.zeros_like(Vbar)
    cbar = None
    for t in range(T - 1, -1, -1):
        S = Vbar @ Df
        if etabar is not None:
            etabar = etabar + (S * Rs[:, t].float()).sum((1, 2)) - lam * Vbar.sum((1, 2))
        Dbar = Dbar + e * (Vbar.transpose(1, 2) @ Rs[:, t].float() - Ys[:, t].float().transpose(1, 2) @ S)
        Yb = Vbar - e * (S @ Dt)
        if t >= 1:
            Vbar = ((1 + mom[t - 1]) * Yb - mom[t] * Ynext) * (As[:, t - 1] > 0)
        else:
            cbar = Yb - mom[0] * Ynext
        Ynext = Yb
    return Dbar, cbar, etabar


def unrolled_forward_hip(X, D, A0, lam, eta, iters, mom=None):
    """Direct-form HIP solve of ``iters`` iterations saving the bf16 slabs; returns
    (R fp32 [G, B, d], D bf16, Y slab, Res slab, A slab)."""
    G, n, d = D.shape
    B = A0.shape[-2]
    dev = D.device
    mom = momentum_schedule(max(iters, 1)) if mom is None else mom
    # the solver reads X per model ([G][B][d])
    Xb = (X if X.dim() == 3 else X.expand(G, B, X.shape[-1])).to(torch.bfloat16).contiguous()
    if tuple(Xb.shape) != (G, B, d):
        raise ValueError(f"X shape {tuple(X.shape)} does not match {(B, d)} or {(G, B, d)}")
    Db = D.to(torch.bfloat16).contiguous()
    Dtb = Db.transpose(1, 2).reshape(G, d // 16, 16, n // 32, 4, 8).permute(0, 1, 3, 4, 2, 5).contiguous()
    Dfb = Db.view(G, n // 16, 16, d // 32, 4, 8).permute(0, 1, 3, 4, 2, 5).contiguous()
    T = max(iters, 1)
    Ys = torch.empty(G, T, B, n, device=dev, dtype=torch.bfloat16)
    Rs = torch.empty(G, T, B, d, device=dev, dtype=torch.bfloat16)
    As = torch.empty(G, T, B, n, device=dev, dtype=torch.bfloat16)
    A = torch.empty(G, B, n, device=dev)
    R = torch.empty(G, B, d, device=dev)
    a0 = A0.float().contiguous()
    if tuple(a0.shape) != (G, B, n):
        raise ValueError(f"A0 shape {tuple(A0.shape)} != {(G, B, n)}")
    mom_d = mom.to(dev)
    rc = _lib.lib().sc_fista(_lib.ptr(Xb), _lib.ptr(Dfb), _lib.ptr(Dtb), _lib.ptr(a0), _lib.ptr(eta),
                             _lib.ptr(lam), _lib.ptr(mom_d), _lib.ptr(A), _lib.ptr(R), G, B, n, d, iters,
                             _lib.ptr(Ys), _lib.ptr(Rs), _lib.ptr(As), _lib.stream_handle(), 0)
    _lib.check(rc, "sc_fista (saving iterates)")
    return R, Db, Ys, Rs, As


def _gram_operands(Xb, Db):
    """C = X D^T (fp32 [G, B, n]) and Gm = D D^T (bf16 [G, n, n], plus its MFMA-fragment-order
    copy the Gram kernel streams)."""
    from . import gemm

    G, n, d = Db.shape
    B = Xb.shape[-2]
    C = torch.empty(G, B, n, device=Db.device)
    gemm.matmul_nt(Xb, Db, C)
    Gm = torch.empty(G, n, n, device=Db.device, dtype=torch.bfloat16)
    gemm.matmul_nt(Db, Db, Gm)
    Gmf = Gm.view(G, n // 16, 16, n // 32, 4, 8).permute(0, 1, 3, 4, 2, 5).contiguous()
    return C, Gm, Gmf


def unrolled_forward_gram(X, D, A0, lam, eta, iters, mom=None):
    """Gram-form HIP solve of ``iters`` iterations (Y += eta (C - Y Gm), one [B, n] x [n, n]
    product per iteration) saving the bf16 Y / A slabs for ``unrolled_backward_gram``.
    Returns (R = X - A_T D fp32 [G, B, d], state for the backward)."""
    from . import gemm

    G, n, d = D.shape
    B = A0.shape[-2]
    dev = D.device
    mom = momentum_schedule(max(iters, 1)) if mom is None else mom
    Xb = X.to(torch.bfloat16).contiguous()
    Db = D.to(torch.bfloat16).contiguous()
    C, Gm, Gmf = _gram_operands(Xb, Db)
    T = int(iters)
    Ys = torch.empty(G, T, B, n, device=dev, dtype=torch.bfloat16)
    As = torch.empty(G, T, B, n, device=dev, dtype=torch.bfloat16)
    Qs = torch.empty(G, T, B, n, device=dev, dtype=torch.bfloat16)
    A = torch.empty(G, B, n, device=dev)
    a0 = A0.float().contiguous()
    if tuple(a0.shape) != (G, B, n):
        raise ValueError(f"A0 shape {tuple(A0.shape)} != {(G, B, n)}")
    rc = _lib.lib().sc_fista_gram(_lib.ptr(C), _lib.ptr(Gmf), _lib.ptr(a0), _lib.ptr(eta), _lib.ptr(lam),
                                  _lib.ptr(mom.to(dev)), _lib.ptr(A), G, B, n, T, _lib.stream_handle(), 0, 1,
                                  _lib.ptr(Ys), _lib.ptr(As), None, _lib.ptr(Qs), None)
    _lib.check(rc, "sc_fista_gram (saving iterates)")
    # R = X - A_T D from the bf16 A_T in the last A slot (the direct form also multiplies bf16 A)
    AD = torch.empty(G, B, d, device=dev)
    _strided_mm(gemm.EPI_F32, 1, B, d, n, As[:, T - 1], n, T * B * n, Db, d, n * d, AD, d, B * d, 1.0)
    R = (X.float() if X.dim() == 3 else X.float().expand(G, B, d)) - AD
    return R, (Xb, Db, Gm, Gmf, Ys, As, Qs)


def unrolled_backward_gram(Rbar, state, eta, mom, T, lam=None, rows: int = 0):
    """Adjoint of ``unrolled_forward_gram``: the reverse sweep runs in the Gram kernel (mode 2:
    Vbar_t in registers, Yb = Vbar - eta Vbar Gm, the support of A_t from the slab), writing the
    Vbar slab and sum_t Vbar_t.  The dictionary gradient then needs no residual slabs:
        Dbar = eta (Vsum^T X - (M + M^T) D) - A_T^T Rbar,   M = sum_t Vbar_t^T Y_t
    (one K = T B GEMM, [n, n] out).  The eta gradient, sum_t <Vbar_t, Q_t> - lam sum Vbar_t with
    Q_t = C - Y_t Gm the forward's step direction (saved as a bf16 slab: from C and Y_t Gm
    separately it would be a difference of terms ~10x its size -- the bf16 GEMM identity
    <Vsum^T X, D> - <M, Gm> is off by ~10%), is accumulated in fp32 inside the sweep.
    ``rows``: 16 / 32 forces the workgroup height.
    Returns (Dbar fp32 [G, n, d], cbar fp32 [G, B, n], etabar [G] or None)."""
    from . import gemm

    Xb, Db, Gm, Gmf, Ys, As, Qs = state
    G, n, d = Db.shape
    B = Ys.shape[2]
    dev = Db.device
    Rb = Rbar.to(torch.bfloat16)
    Rb = (Rb if Rb.dim() == 3 else Rb.expand(G, B, d)).contiguous()
    T2 = torch.empty(G, B, n, device=dev)
    gemm.matmul_nt(Rb, Db, T2)                                     # Rbar D^T
    Vs = torch.empty(G, T, B, n, device=dev, dtype=torch.bfloat16)
    V0 = torch.empty(G, B, n, device=dev)
    stream = _lib.stream_handle()
    _lib.check(_lib.lib().sc_fista_adjoint_init(_lib.ptr(T2), _lib.ptr(V0), _lib.ptr(As), _lib.ptr(Vs), G, B, n, T,
                                                stream), "sc_fista_adjoint_init")
    cbar = torch.empty(G, B, n, device=dev)
    Vsum = torch.empty(G, B, n, device=dev)
    epart = torch.zeros(G, B // 16, device=dev)  # per-workgroup partials (16- or 32-row workgroups)
    lam_t = lam if lam is not None else torch.zeros(G, device=dev)
    rc = _lib.lib().sc_fista_gram(None, _lib.ptr(Gmf), _lib.ptr(V0), _lib.ptr(eta), _lib.ptr(lam_t),
                                  _lib.ptr(torch.as_tensor(mom, dtype=torch.float32).to(dev)), _lib.ptr(cbar), G, B, n,
                                  T, stream, rows, 2, _lib.ptr(Vs), _lib.ptr(As), _lib.ptr(Vsum), _lib.ptr(Qs),
                                  _lib.ptr(epart))
    _lib.check(rc, "sc_fista_gram (adjoint)")
    # M = sum_t Vbar_t^T Y_t: G (n/256)^2 output tiles over K = T B -> split K to fill the chip
    tiles = G * ((n + 255) // 256) ** 2
    ks = 1
    while ks < 16 and tiles * ks * 2 <= 512 and (T * B) % (64 * ks * 2) == 0:
        ks *= 2
    segs = [[(Vs.view(G, T * B, n), Ys.view(G, T * B, n))]]
    if ks > 1:
        slabs = torch.empty(ks, G, n, n, device=dev)
        gemm.weight_grads(segs, [slabs], 1.0, ksplit=ks)
        M = slabs.sum(dim=0)
    else:
        M = torch.empty(G, n, n, device=dev)
        gemm.weight_grads(segs, [M], 1.0)
    VX = torch.empty(G, n, d, device=dev)
    gemm.weight_grads([[(Vsum.to(torch.bfloat16), Xb)]], [VX], 1.0)
    AR = torch.empty(G, n, d, device=dev)
    gemm.weight_grads([[(As[:, T - 1].contiguous(), Rb)]], [AR], 1.0)
    Q = torch.empty(G, n, d, device=dev)
    gemm.matmul_nn((M + M.transpose(1, 2)).to(torch.bfloat16), Db, Q)
    e = eta[:, None, None]
    Dbar = (VX - Q) * e - AR
    etabar = None
    if lam is not None:
        etabar = epart.sum(1) - lam * Vsum.sum((1, 2))
    return Dbar, cbar, etabar


def _gram_unrolled_ok(D, A0) -> bool:
    """The Gram form pays for n <= d (2 B n^2 per iteration and a T B n^2 dictionary-gradient
    GEMM against 4 B n d and 2 T B n d for the direct form)."""
    G, n, d = D.shape
    B = A0.shape[-2]
    return n in GRAM_N and n <= d and B % 128 == 0 and d % 256 == 0


def _strided_mm(epi, layout, M, N, K, a, lda, sa, b, ldb, sb, out, ldc, sc, alpha):
    from . import gemm

    G = b.shape[0]
    gemm._launch(epi, layout, M, N, K, 0, G, [gemm._op(a, lda, sa)] * 2, [gemm._op(b, ldb, sb)] * 2, [out],
                 [alpha], ldc, sc)


def unrolled_backward_hip(Rbar, Db, Ys, Rs, As, eta, mom, T, lam=None):
    """Adjoint sweep on the kernels; returns (Dbar, cbar, etabar) -- etabar (when ``lam`` is
    given) = sum_t <S_t, Res_t> - lam sum Vbar_t from the saved slabs (nS_t = -S_t in Ss)."""
    from . import gemm

    G, n, d = Db.shape
    B = Ys.shape[2]
    dev = Db.device
    Rb = Rbar.to(torch.bfloat16)
    Rb = (Rb if Rb.dim() == 3 else Rb.expand(G, B, d)).contiguous()
    if tuple(Rb.shape) != (G, B, d) or tuple(Ys.shape) != (G, T, B, n) or tuple(Rs.shape) != (G, T, B, d):
        raise ValueError("unrolled FISTA backward: slab / gradient shapes disagree")
    T2 = torch.empty(G, B, n, device=dev)
    gemm.matmul_nt(Rb, Db, T2)                                   # Rbar D^T
    Vs = torch.empty(G, T, B, n, device=dev, dtype=torch.bfloat16)
    Ss = torch.empty(G, T, B, d, device=dev, dtype=torch.bfloat16)
    Vbar = torch.empty(G, B, n, device=dev)
    Ya, Yb_ = torch.zeros(G, B, n, device=dev), torch.empty(G, B, n, device=dev)
    cbar = torch.empty(G, B, n, device=dev)
    stream = _lib.stream_handle()
    _lib.check(_lib.lib().sc_fista_adjoint_init(_lib.ptr(T2), _lib.ptr(Vbar), _lib.ptr(As), _lib.ptr(Vs), G, B, n,
                                                T, stream), "sc_fista_adjoint_init")
    EPI_F32, EPI_BF16 = gemm.EPI_F32, gemm.EPI_BF16
    for t in range(T - 1, -1, -1):
        # nS_t = -(Vbar_t D) into slab slot t, then T2 = nS_t D^T
        _strided_mm(EPI_BF16, 1, B, d, n, Vs[:, t], n, T * B * n, Db, d, n * d, Ss[:, t], d, T * B * d, -1.0)
        _strided_mm(EPI_F32, 3, B, n, d, Ss[:, t], d, T * B * d, Db, d, n * d, T2, n, B * n, 1.0)
        _lib.check(_lib.lib().sc_fista_adjoint(_lib.ptr(T2), _lib.ptr(Vbar), _lib.ptr(Ya), _lib.ptr(Yb_),
                                               _lib.ptr(As), _lib.ptr(Vs), _lib.ptr(cbar), _lib.ptr(eta),
                                               float(mom[t - 1]) if t >= 1 else 0.0, float(mom[t]), G, B, n, T,
                                               t, stream), "sc_fista_adjoint")
        Ya, Yb_ = Yb_, Ya
    # Dbar = eta sum_t (Vbar_t^T Res_t + Y_t^T nS_t) - A_T^T Rbar: one K = T B GEMM + one K = B GEMM
    Dbar = torch.empty(G, n, d, device=dev)
    # G (n/256)(d/256) output tiles over a K = T B reduction: few tiles (32 for 8 models at
    # d = n = 512), so split K until the machine is full; the slabs are summed after
    tiles = G * ((n + 255) // 256) * ((d + 255) // 256)
    ks = 1
    while ks < 16 and tiles * ks * 2 <= 512 and (T * B) % (64 * ks * 2) == 0:
        ks *= 2
    segs = [[(Vs.view(G, T * B, n), Rs.view(G, T * B, d)), (Ys.view(G, T * B, n), Ss.view(G, T * B, d))]]
    if ks > 1:
        slabs = torch.empty(ks, G, n, d, device=dev)
        gemm.weight_grads(segs, [slabs], 1.0, ksplit=ks)
        torch.sum(slabs, dim=0, out=Dbar)
    else:
        gemm.weight_grads(segs, [Dbar], 1.0)
    Dfin = torch.empty(G, n, d, device=dev)
    gemm.weight_grads([[(As[:, T - 1].contiguous(), Rb)]], [Dfin], -1.0)
    Dbar.mul_(eta[:, None, None]).add_(Dfin)
    etabar = None
    if lam is not None:
        etabar = torch.zeros(G, device=dev)
        for t in range(T):  # slab by slab (fp32 temporaries of one iterate, not of all T)
            etabar -= (Ss[:, t].float() * Rs[:, t].float()).sum((1, 2))
            etabar -= lam * Vs[:, t].float().sum((1, 2))
    return Dbar, cbar, etabar


# --------------------------------------------------------------------- direct coefficient search
def coef_search_torch(X, D, lam, lr, iters=100, momentum=0.9, A0=None):
    """Projected SGD with momentum on the codes (reference autoencoders/direct_coef_search.py:
    52-56): grad = 2/(B d) (c D - x) D^T + lam/B sign(c); buf = m buf + grad; c = relu(c - lr buf).
    Batched over models: D [G, n, d], X [B, d] or [G, B, d], lam / lr [G]."""
    D = D.float()
    G, n, d = D.shape
    B = X.shape[-2]
    Xf = X.float()
    lam = torch.as_tensor(lam, dtype=torch.float32, device=D.device).reshape(-1, 1, 1)
    lr = torch.as_tensor(lr, dtype=torch.float32, device=D.device).reshape(-1, 1, 1)
    c = torch.zeros(G, B, n, device=D.device) if A0 is None else A0.float().clone()
    buf = torch.zeros_like(c)
    Dt = D.transpose(1, 2)
    for _ in range(iters):
        grad = 2.0 / (B * d) * (c @ D - Xf) @ Dt + lam / B * torch.sign(c)
        buf = momentum * buf + grad
        c = torch.relu(c - lr * buf)
    return c


def coef_search(X, D, lam, lr, iters: int = 100, momentum: float = 0.9, A0=None, backend: str = "auto"):
    """Direct coefficient search for every model at once; the GPU path is the persistent
    direct-form solver in its projected-momentum mode (one launch for all models and steps,
    bf16 MFMA products, fp32 codes and momentum)."""
    D = D if D.dim() == 3 else D[None]
    G, n, d = D.shape
    B = X.shape[-2]
    ok = (backend != "torch" and _hip_ok(D) and B % 16 == 0 and n % 128 == 0 and d % 128 == 0
          and (d // 128, n // 128) in DIRECT_TILES)
    if backend == "hip" and not ok:
        raise ValueError(f"coef_search HIP path needs B % 16 == 0 and (d/128, n/128) in {sorted(DIRECT_TILES)}")
    if not ok:
        return coef_search_torch(X, D, lam, lr, iters, momentum, A0)
    dev = D.device
    Xb = (X if X.dim() == 3 else X.expand(G, B, d)).to(torch.bfloat16).contiguous()
    if tuple(Xb.shape) != (G, B, d):
        raise ValueError(f"X shape {tuple(X.shape)} does not match {(B, d)} or {(G, B, d)}")
    Db = D.to(torch.bfloat16).contiguous()
    Dtb = Db.transpose(1, 2).reshape(G, d // 16, 16, n // 32, 4, 8).permute(0, 1, 3, 4, 2, 5).contiguous()
    Dfb = Db.view(G, n // 16, 16, d // 32, 4, 8).permute(0, 1, 3, 4, 2, 5).contiguous()
    lam_t = torch.as_tensor(lam, dtype=torch.float32, device=dev).reshape(-1).expand(G).contiguous()
    lr_t = torch.as_tensor(lr, dtype=torch.float32, device=dev).reshape(-1).expand(G).contiguous()
    mom = torch.full((max(iters, 1),), float(momentum), device=dev)
    a0 = None if A0 is None else A0.float().contiguous()
    if a0 is not None and tuple(a0.shape) != (G, B, n):
        raise ValueError(f"A0 shape {tuple(A0.shape)} != {(G, B, n)}")
    A = torch.empty(G, B, n, device=dev)
    rc = _lib.lib().sc_coef_search(_lib.ptr(Xb), _lib.ptr(Dfb), _lib.ptr(Dtb), _lib.ptr(a0), _lib.ptr(lr_t),
                                   _lib.ptr(lam_t), _lib.ptr(mom), _lib.ptr(A), None, G, B, n, d, iters,
                                   2.0 / (B * d), 1.0 / B, _lib.stream_handle())
    _lib.check(rc, "sc_coef_search")
    return A
