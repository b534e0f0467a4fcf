"""A native RCCL communicator on the engine's own HIP streams (graph-capturable collectives).

``torch.distributed``'s ProcessGroupNCCL issues every collective from the host on its internal
stream and tracks it with a watchdog, so the data-parallel steps had to replay their HIP graphs
around host-issued collectives (a replay boundary per collective).  ``RcclComm`` drives the RCCL
C API directly (the same ``librccl`` instance torch loaded, through ctypes -- no second RCCL in the
process): one communicator per process group, created from a unique id that rank 0 draws and the
bootstrap store distributes, and collectives enqueued on a stream the caller chooses.  Enqueued
during ``torch.cuda.graph`` capture they become nodes of the graph: a whole multi-step
data-parallel step (compute, reduce-scatter / all-reduce / all-gather on a side stream, update)
replays as ONE graph (``parallel/graphed.py``).

Reference: the DDP experiment's implicit NCCL all-reduce (``experiments/huge_batch_size.py:274,
313``) and the SURVEY's comm-backend item B3 (an RCCL communicator from a unique id over the
bootstrap store, explicit streams).
"""

from __future__ import annotations

import ctypes as C
import os
from pathlib import Path
from typing import Optional

import torch
import torch.distributed as dist

from .dist import DistInfo

_NCCL_DTYPES = {torch.int8: 0, torch.uint8: 1, torch.int32: 2, torch.int64: 4, torch.float16: 6,
                torch.float32: 7, torch.float64: 8, torch.bfloat16: 9}
NCCL_SUM = 0
_lib = None


class _UniqueId(C.Structure):
    _fields_ = [("internal", C.c_char * 128)]


class RcclError(RuntimeError):
    pass


def library():
    """torch's own librccl (already mapped by ProcessGroupNCCL / torch.cuda.nccl): one RCCL per process."""
    global _lib
    if _lib is None:
        path = Path(torch.__file__).resolve().parent / "lib" / "librccl.so"
        lib = C.CDLL(str(path) if path.exists() else "librccl.so", mode=C.RTLD_GLOBAL)
        vp, sz, i = C.c_void_p, C.c_size_t, C.c_int
        sig = {
            "ncclGetUniqueId": [C.POINTER(_UniqueId)],
            "ncclCommInitRank": [C.POINTER(vp), i, _UniqueId, i],
            "ncclCommDestroy": [vp],
            "ncclAllReduce": [vp, vp, sz, i, i, vp, vp],
            "ncclReduceScatter": [vp, vp, sz, i, i, vp, vp],
            "ncclAllGather": [vp, vp, sz, i, vp, vp],
            "ncclBroadcast": [vp, vp, sz, i, i, vp, vp],
            "ncclAllToAll": [vp, vp, sz, i, vp, vp],
            "ncclGroupStart": [],
            "ncclGroupEnd": [],
            "ncclGetVersion": [C.POINTER(i)],
            "ncclCommCount": [vp, C.POINTER(i)],
            "ncclCommCuDevice": [vp, C.POINTER(i)],
            "ncclCommUserRank": [vp, C.POINTER(i)],
        }
        for name, args in sig.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = C.c_int
        lib.ncclGetErrorString.argtypes = [C.c_int]
        lib.ncclGetErrorString.restype = C.c_char_p
        _lib = lib
    return _lib


def uid_bytes(uid: _UniqueId) -> bytes:
    """All 128 bytes of a unique id (NULs included) for the bootstrap broadcast."""
    return C.string_at(C.addressof(uid), C.sizeof(uid))


def uid_from_bytes(data: bytes) -> _UniqueId:
    if len(data) != C.sizeof(_UniqueId):
        raise RcclError(f"RCCL unique id has {len(data)} bytes, expected {C.sizeof(_UniqueId)}")
    uid = _UniqueId()
    C.memmove(C.addressof(uid), data, len(data))
    return uid


def _check(rc: int, what: str):
    if rc != 0:
        msg = library().ncclGetErrorString(rc)
        raise RcclError(f"{what} failed: {msg.decode() if msg else rc}")


def version() -> int:
    v = C.c_int()
    _check(library().ncclGetVersion(C.byref(v)), "ncclGetVersion")
    return v.value


class RcclComm:
    """One RCCL communicator over the ranks of the default process group.

    ``stream``: the HIP stream collectives run on (default: a new high-priority stream owned by
    this communicator); every collective first makes that stream wait for the CURRENT stream (the
    producer) and returns with the current stream waiting for it, unless ``overlap=True`` -- then the
    caller joins later with ``join()`` (the overlap window).  All of it is capturable."""

    def __init__(self, info: DistInfo, stream: Optional[torch.cuda.Stream] = None):
        if not dist.is_initialized() and info.world_size > 1:
            raise RuntimeError("RcclComm needs the default process group (bootstrap store)")
        self.info = info
        self.world, self.rank = max(1, info.world_size), info.rank
        self.device = torch.device(info.device)
        uid = _UniqueId()
        if self.rank == 0:
            _check(library().ncclGetUniqueId(C.byref(uid)), "ncclGetUniqueId")
        if self.world > 1 or dist.is_initialized():
            # the unique id travels over the bootstrap (the default group's store / collectives).
            # Raw 128 bytes through the struct's address: the ``internal`` field reads back as a
            # bytes COPY cut at the first NUL (and writing through that copy corrupted the heap)
            obj = [uid_bytes(uid) if self.rank == 0 else None]
            dist.broadcast_object_list(obj, src=0, device=self.device if info.backend == "nccl" else None)
            uid = uid_from_bytes(obj[0])
        self._comm = C.c_void_p()
        with torch.cuda.device(self.device):
            _check(library().ncclCommInitRank(C.byref(self._comm), self.world, uid, self.rank), "ncclCommInitRank")
        self.stream = stream or torch.cuda.Stream(self.device, priority=-1)

    # ------------------------------------------------------------------ stream plumbing
    def _enter(self):
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        return cur

    def join(self, stream: Optional[torch.cuda.Stream] = None):
        """Make ``stream`` (default: the current stream) wait for every collective enqueued so far."""
        (stream or torch.cuda.current_stream(self.device)).wait_stream(self.stream)

    def _run(self, fn, overlap: bool, fork: bool = True):
        """Enqueue ``fn(stream)`` after the current stream's work.  ``overlap``: return an event
        recorded right after it on the comm stream (the consumer waits on exactly that op with
        ``torch.cuda.current_stream().wait_event(ev)``); otherwise the current stream waits now.
        ``fork=False``: do not make the comm stream wait for the current stream again -- for the 2nd..
        collectives of a batch issued back to back with no work on the current stream in between (the
        first call's fork already orders them).  Under HIP graph capture on ROCm 7 (MI355X) the first
        current-stream node after MORE than two consecutive forks lost its dependency on the nodes
        before them and ran unordered across graph replays (profiles/r6/graph_capture/README.md), so
        batches fork once."""
        cur = torch.cuda.current_stream(self.device)
        if fork:
            self.stream.wait_stream(cur)
        fn(self.stream.cuda_stream)
        if not overlap:
            cur.wait_stream(self.stream)
            return None
        ev = torch.cuda.Event()
        ev.record(self.stream)
        return ev

    @staticmethod
    def _dt(t: torch.Tensor) -> int:
        if t.dtype not in _NCCL_DTYPES:
            raise TypeError(f"RCCL dtype {t.dtype} not supported")
        if not t.is_contiguous():
            raise ValueError("RCCL buffers must be contiguous")
        return _NCCL_DTYPES[t.dtype]

    # ------------------------------------------------------------------ collectives
    def all_reduce(self, t: torch.Tensor, overlap: bool = False, fork: bool = True):
        """In-place SUM over ranks."""
        dt = self._dt(t)
        return self._run(lambda s: _check(library().ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), dt, NCCL_SUM,
                                                           self._comm, s), "ncclAllReduce"), overlap, fork)

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, overlap: bool = False, fork: bool = True):
        """out = this rank's 1/N block of the SUM of ``inp`` over ranks (inp.numel() == N out.numel())."""
        if inp.numel() != self.world * out.numel() or inp.dtype != out.dtype:
            raise ValueError("reduce_scatter: inp must hold world x out elements of the same dtype")
        dt = self._dt(out)
        self._dt(inp)
        return self._run(lambda s: _check(library().ncclReduceScatter(inp.data_ptr(), out.data_ptr(), out.numel(), dt,
                                                               NCCL_SUM, self._comm, s), "ncclReduceScatter"), overlap, fork)

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, overlap: bool = False, fork: bool = True):
        """out = concat over ranks of ``inp`` (rank-major); ``inp`` may be out's own block (in place)."""
        if out.numel() != self.world * inp.numel() or inp.dtype != out.dtype:
            raise ValueError("all_gather: out must hold world x inp elements of the same dtype")
        dt = self._dt(out)
        return self._run(lambda s: _check(library().ncclAllGather(inp.data_ptr(), out.data_ptr(), inp.numel(), dt,
                                                           self._comm, s), "ncclAllGather"), overlap, fork)

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, overlap: bool = False, fork: bool = True):
        """out[j] = rank j's inp block for this rank (N equal blocks)."""
        if out.numel() != inp.numel() or inp.numel() % self.world or inp.dtype != out.dtype:
            raise ValueError("all_to_all: equal-size buffers of N blocks")
        dt = self._dt(out)
        return self._run(lambda s: _check(library().ncclAllToAll(inp.data_ptr(), out.data_ptr(), inp.numel() // self.world,
                                                          dt, self._comm, s), "ncclAllToAll"), overlap, fork)

    def broadcast(self, t: torch.Tensor, root: int = 0, overlap: bool = False, fork: bool = True):
        dt = self._dt(t)
        return self._run(lambda s: _check(library().ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), dt, int(root),
                                                           self._comm, s), "ncclBroadcast"), overlap, fork)

    # ------------------------------------------------------------------ introspection
    def _query(self, fn: str) -> int:
        v = C.c_int()
        _check(getattr(library(), fn)(self._comm, C.byref(v)), fn)
        return v.value

    def count(self) -> int:
        """Ranks in the communicator, as RCCL itself reports them (ncclCommCount)."""
        return self._query("ncclCommCount")

    def device_index(self) -> int:
        """The HIP device this rank's communicator runs on (ncclCommCuDevice)."""
        return self._query("ncclCommCuDevice")

    def user_rank(self) -> int:
        return self._query("ncclCommUserRank")

    def close(self):
        """Synchronise the device (no captured or enqueued collective may still reference the
        communicator), then destroy it.  Idempotent.  Owners of captured graphs drop them first."""
        if self._comm:
            torch.cuda.synchronize(self.device)
            _check(library().ncclCommDestroy(self._comm), "ncclCommDestroy")
            self._comm = C.c_void_p()

    def __del__(self):  # pragma: no cover - best effort at interpreter exit
        try:
            if self._comm and os.environ.get("SC_RCCL_NO_DESTROY") is None:
                torch.cuda.synchronize(self.device)
                library().ncclCommDestroy(self._comm)
                self._comm = C.c_void_p()
        except Exception:
            pass
