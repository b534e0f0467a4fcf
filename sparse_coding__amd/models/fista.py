"""FISTA dictionary learning (the fork's core; reference ``autoencoders/fista.py``).

* ``FunctionalFista`` -- untied-SAE parameters + a ``hessian_diag`` buffer.  ``loss`` is the
  untied SAE loss (reference :60-84).  After every Adam step the trainer calls
  ``dictionary_update``: FISTA sparse coding warm-started from the encoder's codes
  (500 iterations), an EMA of the Hessian diagonal mean_b(A^2), and a
  Hessian-preconditioned basis step (reference :88-96, big_sweep.py:176-198).
* ``loss2`` -- the "FISTA in the loss" variant (reference :141-172): tied normalised
  SAE loss plus the residual of 50 unrolled FISTA iterations warm-started from c, so
  gradients flow through the solver.  Broken as shipped (B#11); here with identity
  centering.
* ``Fista`` -- the LearnedDict class two of the three shipped checkpoints pickle
  (reference :208-301).

``FistaDictUpdater`` is the batched engine version: one HIP launch solves FISTA for
all models of the ensemble (``ops.fista``), the basis update is batched too.
Reference quirks are reproducible via flags: ``persist_hessian=False`` (B#3: the
EMA is written to a throwaway dict, so H = mean(A^2)/300 every step) and
``normalize="column"`` (B#4: ``norm(2, 0)``).
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch

from ..ops import fista as fista_ops
from .learned_dict import UntiedSAE, _CenteredTied
from .signatures import DictSignature, FunctionalSAE, relu_code, unit_rows, xavier

ACT_HISTORY_LEN = 300


class FunctionalFista(DictSignature):
    fused_kind = "untied"

    @staticmethod
    def init(activation_size, n_dict_components, l1_alpha, bias_decay=0.0, device=None, dtype=None):
        params, buffers = FunctionalSAE.init(activation_size, n_dict_components, l1_alpha, bias_decay, device, dtype)
        buffers["hessian_diag"] = torch.zeros(n_dict_components, device=device)
        return params, buffers

    @staticmethod
    def to_learned_dict(params, buffers):
        return UntiedSAE(params["encoder"], params["decoder"], params["encoder_bias"])

    encode = staticmethod(FunctionalSAE.encode)
    loss = staticmethod(FunctionalSAE.loss)

    # ----------------------------------------------------------------- single-model API
    @staticmethod
    def fista(batch, learned_dict, l1_coef, coefficients, num_iter, device=None, eta=None, threshold=1e-4):
        """Reference signature (:99); returns (ahat, Res).  ``threshold`` is unused, as upstream."""
        eta_t = None if eta is None else torch.as_tensor([float(eta)], device=learned_dict.device)
        A, res = fista_ops.fista(batch, learned_dict[None], torch.as_tensor([float(l1_coef)]),
                                 None if coefficients is None else coefficients[None], num_iter, eta_t,
                                 backend="torch")
        return A[0], res[0]

    @staticmethod
    def quadraticBasisUpdate(learned_dict, Res, ahat, lowestActivation, HessianDiag, stepSize=0.001,
                             Noneg=False):
        return fista_ops.quadratic_basis_update(learned_dict[None], Res[None], ahat[None], HessianDiag[None],
                                                lowestActivation, stepSize, Noneg, normalize="column")[0]

    @staticmethod
    def dictionary_update(params, buffers, batch_centered, coeffs, learned_dict, num_iter=500,
                          persist_hessian=True, normalize="column"):
        """FISTA -> Hessian EMA -> basis update for one model (reference :88-96)."""
        A, res = FunctionalFista.fista(batch_centered, learned_dict, buffers["l1_alpha"], coeffs, num_iter)
        H = fista_ops.hessian_ema(buffers["hessian_diag"], A, ACT_HISTORY_LEN)
        if persist_hessian:
            buffers["hessian_diag"] = H
        new = fista_ops.quadratic_basis_update(learned_dict[None], res[None], A[None], H[None], 0.001, 0.001,
                                               normalize=normalize)[0]
        return new, res

    # ----------------------------------------------------------------- FISTA in the loss
    @staticmethod
    def loss2(params, buffers, batch, num_iter: int = 50):
        """Tied normalised SAE loss + |X - FISTA_50(c) D|^2 (differentiable through the solver)."""
        w = unit_rows(params["encoder"])
        c = relu_code(batch, w, params["encoder_bias"])
        xc_hat = c @ w
        l_rec = (xc_hat - batch).pow(2).mean()
        l_l1 = buffers["l1_alpha"] * c.abs().sum(-1).mean()
        l_bd = buffers.get("bias_decay", 0.0) * torch.linalg.vector_norm(params["encoder_bias"])
        res = _unrolled_fista_residual(batch, w, buffers["l1_alpha"], c, num_iter)
        l_fista = res.pow(2).mean()
        total = l_rec + l_fista + l_l1 + l_bd
        return total, ({"loss": total, "l_reconstruction": l_rec, "l_fista": l_fista, "l_l1": l_l1}, {"c": c})

    @staticmethod
    def fista_loss(params, buffers, batch, c, num_iter: int = 50):
        w = unit_rows(params["encoder"])
        res = _unrolled_fista_residual(batch, w, buffers["l1_alpha"], c, num_iter)
        l = res.pow(2).mean()
        return l, ({"loss": l}, {"c_fista": c})


def _unrolled_fista_residual(X, D, lam, A0, iters, eta=None):
    """Differentiable FISTA residual X - A_T D.  eta = 1 / eigvalsh(D D^T).max() is computed from
    the differentiable dictionary and NOT detached, as upstream (reference fista.py:104-106), so
    the gradient includes the path through the step size.  Plain tensors go through
    ``ops.fista.unrolled_fista_residual`` (explicit adjoint sweep: HIP slabs + MFMA GEMMs on the
    GPU, fp32 torch otherwise); under functorch transforms (``FunctionalEnsemble``'s
    vmap(grad(loss))) the iterations run as plain differentiable torch ops."""
    if eta is None:
        eta = 1.0 / torch.linalg.eigvalsh(D @ D.T).max()
    wrapped = any(torch.is_tensor(t) and torch._C._functorch.is_functorch_wrapped_tensor(t)
                  for t in (X, D, A0, eta, lam))
    if wrapped:
        return fista_ops.unrolled_fista_plain(X, D[None], lam, A0[None], iters, eta)[0]
    R = fista_ops.unrolled_fista_residual(X, D[None], lam, A0[None], iters, eta)
    return R[0]


class Fista(_CenteredTied):
    """Tied-style inference dictionary with centering and its own solver (reference :208-301)."""

    def fista(self, batch, coefficients, device, l1_coef, num_iter, eta=None):
        D = self.get_learned_dict()
        eta_t = None if eta is None else torch.as_tensor([float(eta)], device=D.device)
        A, res = fista_ops.fista(batch, D[None], torch.as_tensor([float(l1_coef)]), coefficients[None],
                                 num_iter, eta_t, backend="torch")
        return A[0], res[0]


@dataclass
class FistaDictUpdater:
    """Batched FISTA dictionary update applied to a stacked ensemble after each Adam step.

    Mirrors the fork's ``ensemble_train_loop`` (big_sweep.py:176-198): codes from the
    encoder warm-start FISTA on the (centered) batch, then the basis update overwrites the
    decoder (Adam moments are kept, as upstream).
    """

    num_iter: int = 500
    persist_hessian: bool = True   # False reproduces B#3
    normalize: str = "column"      # "column" reproduces B#4, "row" = unit-norm atoms
    backend: str = "auto"          # "hip" | "torch" | "auto"
    eta_method: str = "tracked"   # "eigh" = exact per call (reference); "tracked" = warm power
                                  # iteration + exact refresh every 50 calls, 0.1% safe margin
    step: float = 0.001
    lowest_activation: float = 0.001
    hessian: Optional[torch.Tensor] = None
    _eta: Optional[object] = None  # EtaTracker state when eta_method == "tracked"

    def __call__(self, decoder: torch.Tensor, batch: torch.Tensor, codes: torch.Tensor, l1: torch.Tensor):
        """decoder [G, n, d] raw; batch [B, d]; codes [G, B, n]; returns (new decoder, residual, A).

        On the GPU with the Gram-form shapes (``fista_ops.gram_solve_ok``) the step runs the hot path:
        X D^T and D D^T on the MFMA GEMM, eta from the solver's own Gram (``EtaTracker.from_gram``),
        the persistent solve, the residual by the decoder GEMM's epilogue (bf16, negated) and the basis
        update on those bf16 operands -- no fp32 GEMM, no operand copies; the returned residual is then
        the bf16 one (fp32 view)."""
        D = unit_rows(decoder.float())
        if self.backend != "torch" and fista_ops.gram_solve_ok(batch, D):
            tracker = None
            if self.eta_method == "tracked":
                if self._eta is None:
                    self._eta = fista_ops.EtaTracker()
                tracker = self._eta
            eta = None if tracker is not None else fista_ops.step_size(D, self.eta_method)
            A, Ab, Rn, _, _ = fista_ops.gram_solve(batch, D, l1, codes, self.num_iter, eta=eta, tracker=tracker)
            G, n = D.shape[0], D.shape[1]
            H0 = self.hessian if (self.persist_hessian and self.hessian is not None) else torch.zeros(G, n, device=D.device)
            H = fista_ops.hessian_ema(H0, A, ACT_HISTORY_LEN)
            if self.persist_hessian:
                self.hessian = H
            new = fista_ops.quadratic_basis_update(D, None, A, H, self.lowest_activation, self.step,
                                                   normalize=self.normalize, A_bf16=Ab, res_neg_bf16=Rn)
            return new, Rn.float().neg_(), A
        if self.eta_method == "tracked":
            if self._eta is None:
                self._eta = fista_ops.EtaTracker()
            eta = self._eta(D)
        else:
            eta = fista_ops.step_size(D, self.eta_method)
        A, res = fista_ops.fista(batch, D, l1, codes, self.num_iter, eta, backend=self.backend)
        G, n = D.shape[0], D.shape[1]
        H0 = self.hessian if (self.persist_hessian and self.hessian is not None) else torch.zeros(G, n, device=D.device)
        H = fista_ops.hessian_ema(H0, A, ACT_HISTORY_LEN)
        if self.persist_hessian:
            self.hessian = H
        new = fista_ops.quadratic_basis_update(D, res, A, H, self.lowest_activation, self.step,
                                               normalize=self.normalize)
        return new, res, A
