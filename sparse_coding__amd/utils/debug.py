"""Debug and determinism aids (race detection / sanitizers).

GPU AddressSanitizer and XNACK builds are not available on the MI355X pool, so the
checks here are the ones that run on a normal build:

* ``debug_mode()`` -- synchronise after every HIP kernel launch of this package so an
  asynchronous fault is reported at the launch that caused it, and check the named
  tensors for non-finite values after each training step (``check_finite``);
* ``assert_deterministic(make_state, step)`` -- run one step twice from identical state
  and compare every output bit for bit (the GEMM epilogues, bias reduction and top-k
  select are designed to be deterministic; no float atomics on the training path);
* ``serialize_streams()`` -- make the data-parallel collectives (RCCL stream) complete before the
  next kernel is issued, to tell a stream-ordering race from a numerical bug.
"""

from __future__ import annotations

import contextlib
import os
from typing import Callable, Dict, Iterable, Optional

import torch

from ..ops import _lib


@contextlib.contextmanager
def debug_mode(enabled: bool = True):
    old = _lib._DEBUG_SYNC
    _lib.set_debug_sync(enabled)
    try:
        yield
    finally:
        _lib.set_debug_sync(old)


def check_finite(tensors: Dict[str, torch.Tensor], where: str = ""):
    bad = [k for k, t in tensors.items() if torch.is_tensor(t) and t.is_floating_point() and
           not bool(torch.isfinite(t).all())]
    if bad:
        raise FloatingPointError(f"non-finite values in {bad} {where}".strip())


def assert_deterministic(make_state: Callable[[], object], step: Callable[[object], Dict[str, torch.Tensor]]):
    """``make_state()`` builds a fresh engine/state; ``step(state)`` runs it and returns the
    tensors to compare.  Raises if any differ bitwise between two runs."""
    a = step(make_state())
    b = step(make_state())
    diff = [k for k in a if not torch.equal(a[k], b[k])]
    if diff:
        raise AssertionError(f"non-deterministic outputs: {diff}")
    return a


@contextlib.contextmanager
def serialize_streams():
    """No compute / communication overlap: data-parallel collectives complete before the next
    kernel is issued (``parallel.data_parallel.serialized`` checks ``SC_SERIALIZE_STREAMS``)."""
    old = os.environ.get("SC_SERIALIZE_STREAMS")
    os.environ["SC_SERIALIZE_STREAMS"] = "1"
    try:
        yield
    finally:
        if old is None:
            os.environ.pop("SC_SERIALIZE_STREAMS", None)
        else:
            os.environ["SC_SERIALIZE_STREAMS"] = old
