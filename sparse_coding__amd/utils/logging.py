"""Logging / observability.

The reference logs to wandb only (``big_sweep.py:204-228, 353-362``).  Here a
``Logger`` fans out to pluggable sinks -- stdout, a JSONL file (default) and
wandb when it is importable -- and metric names follow the reference
(``{ensemble}_{hparam_name}_{loss_key}``).  ``StepTimer`` measures device time
with HIP events; ``trace_range`` emits roctx ranges (visible in rocprofv3 with
marker tracing) around phases.
"""

from __future__ import annotations

import contextlib
import json
import os
import sys
import time
from typing import Any, Dict, Iterable, List, Optional

import torch


class Sink:
    def log(self, metrics: Dict[str, Any], step: int):
        raise NotImplementedError

    def close(self):
        pass


class StdoutSink(Sink):
    def __init__(self, every: int = 1, stream=sys.stdout):
        self.every = every
        self.stream = stream

    def log(self, metrics, step):
        if step % self.every:
            return
        items = ", ".join(f"{k}={v:.4g}" if isinstance(v, float) else f"{k}={v}" for k, v in list(metrics.items())[:12])
        print(f"[step {step}] {items}", file=self.stream, flush=True)


class JsonlSink(Sink):
    def __init__(self, path: str):
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        self.fh = open(path, "a", buffering=1)

    def log(self, metrics, step):
        rec = {"step": step, "time": time.time()}
        rec.update({k: (float(v) if torch.is_tensor(v) else v) for k, v in metrics.items()})
        self.fh.write(json.dumps(rec) + "\n")

    def close(self):
        self.fh.close()


class WandbSink(Sink):
    def __init__(self, project="sparse coding", entity=None, config=None, name=None):
        import wandb  # optional dependency

        self.run = wandb.init(project=project, entity=entity, config=config, name=name)

    def log(self, metrics, step):
        self.run.log(metrics, step=step)

    def close(self):
        self.run.finish()


class Logger:
    def __init__(self, sinks: Iterable[Sink] = ()):
        self.sinks: List[Sink] = list(sinks)

    @classmethod
    def from_config(cls, log_dir: str = "", use_wandb: bool = False, stdout_every: int = 0, config=None,
                    rank: int = 0):
        sinks: List[Sink] = []
        if rank != 0:
            return cls(sinks)
        if log_dir:
            sinks.append(JsonlSink(os.path.join(log_dir, "metrics.jsonl")))
        if stdout_every:
            sinks.append(StdoutSink(stdout_every))
        if use_wandb:
            try:
                sinks.append(WandbSink(config=config))
            except Exception as e:  # wandb absent offline: keep training, say so once
                print(f"[logger] wandb unavailable ({e}); logging to JSONL/stdout only", file=sys.stderr)
        return cls(sinks)

    def log(self, metrics: Dict[str, Any], step: int):
        for s in self.sinks:
            s.log(metrics, step)

    def close(self):
        for s in self.sinks:
            s.close()


def model_metric_names(ensemble: str, hparams: List[dict], losses: List[Dict[str, float]]) -> Dict[str, float]:
    """Flatten per-model losses as ``{ensemble}_{hparam-name}_{key}`` (reference big_sweep.py:204-228)."""
    from .config import make_hyperparam_name

    out = {}
    for hp, ld in zip(hparams, losses):
        name = make_hyperparam_name(hp)
        for k, v in ld.items():
            out[f"{ensemble}_{name}_{k}"] = v
    return out


class StepTimer:
    """Device-time measurement of a region with HIP events (no host sync until ``elapsed``)."""

    def __init__(self):
        self.enabled = torch.cuda.is_available()
        self.start = torch.cuda.Event(enable_timing=True) if self.enabled else None
        self.end = torch.cuda.Event(enable_timing=True) if self.enabled else None
        self.t0 = 0.0

    def __enter__(self):
        if self.enabled:
            self.start.record()
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        if self.enabled:
            self.end.record()
        self.t1 = time.perf_counter()

    def elapsed_ms(self) -> float:
        if self.enabled:
            self.end.synchronize()
            return self.start.elapsed_time(self.end)
        return (self.t1 - self.t0) * 1e3


@contextlib.contextmanager
def trace_range(name: str):
    """roctx range (torch.cuda.nvtx maps to roctx on ROCm builds); no-op without a GPU."""
    if torch.cuda.is_available():
        torch.cuda.nvtx.range_push(name)
        try:
            yield
        finally:
            torch.cuda.nvtx.range_pop()
    else:
        yield
