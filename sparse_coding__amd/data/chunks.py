"""Activation chunk files in the reference layout, read by the native prefetcher.

Layout (reference ``activation_dataset.py:393-397``): ``{folder}/{i}.pt`` holds one
fp16 tensor ``[rows, d]`` written with ``torch.save``.  Reading goes through
``_sc_runtime.so`` (``csrc/runtime/chunk_reader.cpp``): the zip entry with the raw
storage is located without unpickling and pulled into a pinned host buffer by a
thread pool, asynchronously (``prefetch``), then copied to HBM with a non-blocking
H2D.  Shapes come from ``torch.load(mmap=True, weights_only=True)``, which touches
only the pickle header.
"""

from __future__ import annotations

import ctypes as C
import os
import threading
from pathlib import Path
from typing import List, Optional, Tuple

import torch

_RT = None
_RT_LOCK = threading.Lock()


def runtime():
    """ctypes handle of the native runtime library (built in-tree on first use)."""
    global _RT
    if _RT is not None:
        return _RT
    with _RT_LOCK:
        if _RT is None:
            here = Path(__file__).resolve().parent.parent / "ops"
            path = here / "_sc_runtime.so"
            if not path.exists():
                from ..ops import build

                build.build(verbose=False)
            lib = C.CDLL(str(path))
            lib.sc_zip_find.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
            lib.sc_zip_find.restype = C.c_int
            lib.sc_prefetcher_create.argtypes = [C.c_int]
            lib.sc_prefetcher_create.restype = C.c_void_p
            lib.sc_prefetcher_destroy.argtypes = [C.c_void_p]
            lib.sc_prefetch_submit.argtypes = [C.c_void_p, C.c_char_p, C.c_int64, C.c_int64, C.c_void_p]
            lib.sc_prefetch_submit.restype = C.c_int
            lib.sc_prefetch_wait.argtypes = [C.c_void_p, C.c_int]
            lib.sc_prefetch_wait.restype = C.c_int
            lib.sc_prefetch_poll.argtypes = [C.c_void_p, C.c_int]
            lib.sc_prefetch_poll.restype = C.c_int
            _RT = lib
    return _RT


def storage_extent(path: str) -> Tuple[int, int]:
    """(byte offset, byte size) of the tensor storage inside a torch.save archive."""
    off, size = C.c_int64(), C.c_int64()
    rc = runtime().sc_zip_find(path.encode(), b"/data/0", C.byref(off), C.byref(size))
    if rc != 0:
        raise IOError(f"{path}: not an uncompressed torch.save archive (code {rc})")
    return off.value, size.value


def save_chunk(tensor: torch.Tensor, folder: str, index: int, dtype=torch.float16) -> str:
    """Write ``{folder}/{index}.pt`` exactly like the reference harvester (fp16, contiguous)."""
    os.makedirs(folder, exist_ok=True)
    path = os.path.join(folder, f"{index}.pt")
    t = tensor.detach().to("cpu", dtype).contiguous().clone()
    torch.save(t, path + ".tmp")
    os.replace(path + ".tmp", path)
    return path


class ChunkFolder:
    """Random access to ``{i}.pt`` chunks with asynchronous native prefetch."""

    def __init__(self, folder: str, threads: int = 8):
        self.folder = folder
        files = [f for f in os.listdir(folder) if f.endswith(".pt") and f[:-3].isdigit()]
        self.indices = sorted(int(f[:-3]) for f in files)
        self._pf = runtime().sc_prefetcher_create(threads)
        self._meta = {}

    def __len__(self):
        return len(self.indices)

    def path(self, i: int) -> str:
        return os.path.join(self.folder, f"{i}.pt")

    def meta(self, i: int) -> Tuple[torch.Size, torch.dtype]:
        if i not in self._meta:
            t = torch.load(self.path(i), mmap=True, weights_only=True, map_location="cpu")
            self._meta[i] = (t.shape, t.dtype)
        return self._meta[i]

    def prefetch(self, i: int, pin: bool = True):
        """Start reading chunk ``i``; returns a handle for ``get``."""
        shape, dtype = self.meta(i)
        off, size = storage_extent(self.path(i))
        buf = torch.empty(shape, dtype=dtype, pin_memory=pin and torch.cuda.is_available())
        if size != buf.numel() * buf.element_size():
            return ("eager", i, None)  # storage larger than the tensor (a saved view): plain load
        ticket = runtime().sc_prefetch_submit(self._pf, self.path(i).encode(), off, size, C.c_void_p(buf.data_ptr()))
        return ("native", ticket, buf)

    def get(self, handle) -> torch.Tensor:
        kind, ticket, buf = handle
        if kind == "eager":
            return torch.load(self.path(ticket), weights_only=True, map_location="cpu")
        rc = runtime().sc_prefetch_wait(self._pf, ticket)
        if rc != 0:
            raise IOError("native chunk read failed")
        return buf

    def load(self, i: int, device=None, dtype=None) -> torch.Tensor:
        t = self.get(self.prefetch(i))
        if device is not None or dtype is not None:
            t = t.to(device=device or t.device, dtype=dtype or t.dtype, non_blocking=True)
        return t

    def n_rows(self) -> int:
        return sum(self.meta(i)[0][0] for i in self.indices)

    def __del__(self):
        try:
            if self._pf:
                runtime().sc_prefetcher_destroy(self._pf)
                self._pf = None
        except Exception:
            pass
