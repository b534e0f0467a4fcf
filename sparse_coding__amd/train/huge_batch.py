"""Single large dictionary, data parallel, with dead-feature resampling.

Reference: ``experiments/huge_batch_size.py`` -- an ``nn.Module`` SAE (``SAE``:
tied-init dictionary + separate encoder + learned centering; ``UntiedSAE``) trained
with DDP over gloo (``process_main``), and a single-GPU variant that every 10
chunks re-initialises dead features from the worst-reconstructed examples
(``process_reinit``, ``WorstIndices``).  The reference DDP path does not import
(B#9); this one runs.

MI355X design:

* ``engine="fused"`` (default on GPU): the untied SAE runs on the fused gfx950
  step (``FusedSAEEnsemble`` with G=1) and ``DataParallelFused`` all-reduces its
  gradients over RCCL, overlapped with the second weight-gradient GEMM.  Batches
  are gathered from an HBM ring holding the whole chunk (no DataLoader workers).
* ``engine="torch"``: the reference modules (with learned centering) under
  ``torch.nn.parallel.DistributedDataParallel`` -- the CPU/gloo and parity path.
* resampling is tracked on device: per-feature fire counts come from the encoder
  epilogue (every step), and the worst-reconstructed examples are kept as a device
  top-k over ring indices (``WorstIndices`` without a per-example host loop).  With
  several ranks the resampled rows are computed on rank 0 and broadcast.
"""

from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from ..data.chunks import ChunkFolder
from ..data.ring import DeviceRing
from ..models.learned_dict import LearnedDict
from ..models.signatures import FunctionalSAE
from ..parallel.dist import DistInfo, init_distributed
from ..utils.config import BaseArgs, _default_device
from ..utils.logging import Logger


# ----------------------------------------------------------------------------- reference modules
class HugeSAE(nn.Module, LearnedDict):
    """Reference ``SAE`` (huge_batch_size.py:25-65): unit-row dictionary, encoder init to its
    transpose, ReLU(threshold) codes of the centred input, centring added back."""

    def __init__(self, input_size, latent_size, l1_alpha):
        super().__init__()
        w = torch.randn(latent_size, input_size)
        w = w / w.norm(dim=-1, keepdim=True)
        self.dict = nn.Parameter(w)
        self.encoder = nn.Parameter(w.clone().T)
        self.threshold = nn.Parameter(torch.zeros(latent_size))
        self.centering = nn.Parameter(torch.zeros(input_size))
        self.l1_alpha = l1_alpha
        self.n_feats, self.activation_size = latent_size, input_size

    def dict_param(self) -> nn.Parameter:
        return self.dict

    def get_learned_dict(self):
        w = self.dict_param()
        return w / w.norm(dim=-1, keepdim=True)

    def encode(self, x):
        return F.relu((x - self.centering) @ self.encoder + self.threshold)

    def _decode_offset(self):
        return self.centering

    def forward(self, x):
        c = self.encode(x)
        x_hat = c @ self.get_learned_dict() + self._decode_offset()
        per_ex = (x - x_hat).pow(2).mean(dim=-1)
        mse = per_ex.mean()
        sparsity = self.l1_alpha * c.abs().sum(-1).mean()
        return mse + sparsity, mse, sparsity, c, per_ex

    def to_device(self, device):
        self.to(device)


class HugeUntiedSAE(HugeSAE):
    """Reference ``UntiedSAE`` (huge_batch_size.py:67-101): random encoder, the centring is
    subtracted before encoding but not added back."""

    def __init__(self, input_size, latent_size, l1_alpha):
        super().__init__(input_size, latent_size, l1_alpha)
        self.decoder = nn.Parameter(self.dict.data)  # reference parameter name (state-dict keys)
        del self.dict
        with torch.no_grad():
            self.encoder.copy_(torch.randn(input_size, latent_size))

    def dict_param(self) -> nn.Parameter:
        return self.decoder

    def _decode_offset(self):
        return 0.0


# ----------------------------------------------------------------------------- resampling
class WorstIndices:
    """Device top-k of the largest per-example losses seen (reference :120-146)."""

    def __init__(self, k: int, device):
        self.k = k
        self.loss = torch.full((k,), -float("inf"), device=device)
        self.idx = torch.full((k,), -1, dtype=torch.long, device=device)

    def update(self, idx: torch.Tensor, loss: torch.Tensor):
        all_loss = torch.cat([self.loss, loss.float()])
        all_idx = torch.cat([self.idx, idx.long()])
        top = torch.topk(all_loss, self.k)
        self.loss, self.idx = top.values, all_idx[top.indices]

    def get_worst(self, n: int) -> torch.Tensor:
        valid = self.idx[torch.isfinite(self.loss)]
        return valid[:n]  # topk output is sorted descending


def resample_dead(enc_rows: torch.Tensor, dead: torch.Tensor, worst_vectors: torch.Tensor, adam_rows: List[torch.Tensor],
                  encoder_norm_ratio: float = 0.2) -> int:
    """Re-initialise dead features' encoder rows from the worst examples and zero their Adam
    moments (reference huge_batch_size.py:216-236).  ``enc_rows``: [n, d] view of the
    encoder (feature-major); ``adam_rows``: tensors whose leading axis is the feature axis."""
    n_rep = min(int(dead.numel()), worst_vectors.shape[0])
    if n_rep == 0:
        return 0
    dead = dead[:n_rep]
    av_norm = enc_rows.norm(dim=-1).mean()
    enc_rows[dead] = worst_vectors[:n_rep].to(enc_rows.dtype) * encoder_norm_ratio / av_norm
    for t in adam_rows:
        t[dead] = 0
    return n_rep


# ----------------------------------------------------------------------------- config + driver
@dataclass
class HugeBatchArgs(BaseArgs):
    """Reference HugeBatchArgs / HugeReinitArgs (huge_batch_size.py:348-411)."""

    dataset_folder: str = "activation_data/layer_12"
    output_dir: str = "huge_batch_size"
    batch_size: int = 2048           # per rank
    seed: int = 0
    lr: float = 1e-3
    l1_alpha: float = 1e-3
    n_features: int = 4096
    reinit: bool = False
    reinit_every: int = 10           # chunks
    tied: bool = False               # HugeSAE (learned centring, torch engine) vs untied
    engine: str = "auto"             # auto | fused | torch
    n_epochs: int = 1
    max_steps_per_chunk: int = 0     # 0 = full chunk
    device: str = field(default_factory=_default_device)
    log_every: int = 50


class HugeBatchTrainer:
    def __init__(self, cfg: HugeBatchArgs, d: int, info: Optional[DistInfo] = None):
        self.cfg = cfg
        self.info = info or DistInfo()
        self.device = self.info.device if self.info.device.type == "cuda" else torch.device(cfg.device)
        torch.manual_seed(cfg.seed)
        n = cfg.n_features
        fused_ok = (self.device.type == "cuda" and not cfg.tied and cfg.batch_size % 128 == 0 and n % 128 == 0
                    and d % 256 == 0)
        eng = cfg.engine if cfg.engine != "auto" else ("fused" if fused_ok else "torch")
        if eng == "fused" and not fused_ok:
            raise ValueError("fused engine needs a GPU, an untied SAE and B%128, n%128, d%256 == 0")
        self.engine = eng
        self.d, self.n = d, n
        if eng == "fused":
            from ..engine.fused import FusedSAEEnsemble
            from ..parallel.data_parallel import DataParallelFused

            models = [FunctionalSAE.init(d, n, cfg.l1_alpha)]
            self.impl = FusedSAEEnsemble(models, FunctionalSAE, lr=cfg.lr, batch_size=cfg.batch_size,
                                         device=self.device, count_every=1)
            self.dp = DataParallelFused(self.impl, self.info)
        else:
            self.module = (HugeSAE if cfg.tied else HugeUntiedSAE)(d, n, cfg.l1_alpha).to(self.device)
            self.model = self.module
            if self.info.enabled:
                from torch.nn.parallel import DistributedDataParallel as DDP

                self.model = DDP(self.module, device_ids=[self.device.index] if self.device.type == "cuda" else None)
            self.opt = torch.optim.Adam(self.model.parameters(), lr=cfg.lr)
            self.counts = torch.zeros(n, device=self.device)
        self.worst = WorstIndices(n, self.device)
        self.n_samples = 0

    # ------------------------------------------------------------------ one step
    def step(self, x: torch.Tensor, idx: torch.Tensor):
        if self.engine == "fused":
            out = self.dp.step_batch(x)
            per_ex = self.impl.r[0].float().pow(2).mean(-1)
            mse = out[0, 1]
            loss = out[0, 0]
            l0 = out[0, 4]
        else:
            self.opt.zero_grad(set_to_none=True)
            loss, mse, _, c, per_ex = self.model(x.float())
            loss.backward()
            self.opt.step()
            with torch.no_grad():
                self.counts += (c > 0).sum(0)
            l0 = (c > 0).sum(-1).float().mean()
        if self.cfg.reinit:
            self.worst.update(idx, per_ex.detach())
        self.n_samples += x.shape[0] * self.info.world_size
        return loss, mse, l0

    def feature_counts(self) -> torch.Tensor:
        c = self.impl.feature_counts[0].clone() if self.engine == "fused" else self.counts.clone()
        if self.info.enabled:
            dist.all_reduce(c)
        return c

    def reset_counts(self):
        if self.engine == "fused":
            self.impl.feature_counts.zero_()
        else:
            self.counts.zero_()
        self.worst = WorstIndices(self.n, self.device)

    @torch.no_grad()
    def resample(self, ring: DeviceRing) -> int:
        dead = torch.nonzero(self.feature_counts() == 0).flatten()
        n_dead = int(dead.numel())
        if n_dead and self.info.is_main:
            vecs = ring.buf.index_select(0, self.worst.get_worst(n_dead)).float()
            if self.engine == "fused":
                e = self.impl
                rows = [e.m["encoder"][0], e.v["encoder"][0], e.m["decoder"][0], e.v["decoder"][0],
                        e.m["encoder_bias"][0], e.v["encoder_bias"][0]]
                n_rep = resample_dead(e.params["encoder"][0], dead, vecs, rows)
            else:
                m = self.module
                st = self.opt.state
                rows = []
                for p, t in ((m.dict_param(), False), (m.encoder, True), (m.threshold, False)):
                    if p in st:
                        rows += [st[p]["exp_avg"].T if t else st[p]["exp_avg"],
                                 st[p]["exp_avg_sq"].T if t else st[p]["exp_avg_sq"]]
                n_rep = resample_dead(m.encoder.data.T, dead, vecs, rows)
        if self.info.enabled:
            self._broadcast_state()
        if self.engine == "fused":
            self.impl.refresh_shadows()
        return n_dead

    def _broadcast_state(self):
        if self.engine == "fused":
            e = self.impl
            ts = list(e.params.values()) + list(e.m.values()) + list(e.v.values())
        else:
            ts = [p.data for p in self.module.parameters()]
            for s in self.opt.state.values():
                ts += [s["exp_avg"], s["exp_avg_sq"]]
        for t in ts:
            dist.broadcast(t, src=0)

    # ------------------------------------------------------------------ export
    def state_dict_reference(self):
        """Reference ``UntiedSAE.state_dict()`` layout (decoder [n,d], encoder [d,n], threshold, centering)."""
        if self.engine == "fused":
            e = self.impl
            return {"decoder": e.params["decoder"][0].cpu().clone(), "encoder": e.params["encoder"][0].T.cpu().clone(),
                    "threshold": e.params["encoder_bias"][0].cpu().clone(), "centering": torch.zeros(self.d)}
        return {k: v.detach().cpu().clone() for k, v in self.module.state_dict().items()}


def train(cfg: HugeBatchArgs, info: Optional[DistInfo] = None, logger: Optional[Logger] = None):
    info = info or init_distributed()
    folder = ChunkFolder(cfg.dataset_folder)
    d = folder.meta(folder.indices[0])[0][1]
    tr = HugeBatchTrainer(cfg, d, info)
    rows_max = max(folder.meta(i)[0][0] for i in folder.indices)
    ring_dtype = torch.bfloat16 if tr.engine == "fused" else torch.float32
    ring = DeviceRing(rows_max, d, device=tr.device, dtype=ring_dtype, seed=cfg.seed)
    logger = logger or Logger.from_config(cfg.output_dir, rank=info.rank)
    os.makedirs(cfg.output_dir, exist_ok=True)
    xbuf = torch.empty(cfg.batch_size, d, device=tr.device, dtype=ring_dtype)
    step = 0
    history = []
    for epoch in range(cfg.n_epochs):
        for ci, chunk_idx in enumerate(folder.indices):
            ring.size = ring.head = 0
            ring.push(folder.load(chunk_idx).to(tr.device, non_blocking=True))
            n_batches = ring.size // (cfg.batch_size * info.world_size)
            if cfg.max_steps_per_chunk:
                n_batches = min(n_batches, cfg.max_steps_per_chunk)
            for _ in range(n_batches):
                x, idx = ring.sample_shard(cfg.batch_size, info.rank, info.world_size, out=xbuf, return_index=True)
                loss, mse, l0 = tr.step(x, idx)
                step += 1
                if cfg.log_every and step % cfg.log_every == 0:
                    logger.log({"loss": float(loss.detach()), "mse": float(mse.detach()), "n_nonzero": float(l0),
                                "n_samples": tr.n_samples}, step)
            rec = {"chunk": chunk_idx, "epoch": epoch}
            if cfg.reinit and chunk_idx % cfg.reinit_every == 0:  # reference :204
                rec["n_dead_feats"] = tr.resample(ring)
                tr.reset_counts()
            history.append(rec)
            logger.log(rec, step)
            if info.is_main:
                torch.save(tr.state_dict_reference(), os.path.join(cfg.output_dir, f"sae_{chunk_idx}.pt"))
    logger.close()
    return tr, history


if __name__ == "__main__":
    train(HugeBatchArgs.from_cli())
