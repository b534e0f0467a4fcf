"""ctypes binding to the in-tree gfx950 kernel library (``_sc_kernels.so``).

The library is loaded lazily, after ``torch`` has mapped its HIP runtime.  On a
machine with a GPU the kernels are mandatory: if the library is missing we try
one in-tree build and otherwise raise -- there is no silent eager fallback for
the fused paths.
"""

from __future__ import annotations

import ctypes as C
import os
import threading
from pathlib import Path

import torch

_HERE = Path(__file__).resolve().parent
_LIB_PATH = _HERE / "_sc_kernels.so"
_lock = threading.Lock()
_lib = None

c_int, c_long, c_float, c_void_p = C.c_int, C.c_long, C.c_float, C.c_void_p
c_float_p = C.POINTER(C.c_float)


class ScOperand(C.Structure):
    _fields_ = [("ptr", c_void_p), ("ld", c_long), ("sg", c_long)]


class KernelError(RuntimeError):
    pass


def signatures():
    """(required, optional) C signatures of the kernel library: name -> argument types."""
    sig = {
        "sc_gemm": [c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                    C.POINTER(ScOperand), C.POINTER(ScOperand), C.POINTER(c_void_p), c_float_p,
                    c_long, c_long, c_void_p, c_long, c_void_p, c_void_p, c_long, c_long,
                    c_void_p, c_void_p, c_void_p, c_float,
                    c_void_p, c_int,
                    c_int, c_int, c_long, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                    c_void_p, c_void_p, c_void_p, c_void_p],
        "sc_adam_rows": [c_int, C.POINTER(c_void_p), C.POINTER(c_void_p), C.POINTER(c_void_p),
                         C.POINTER(c_void_p), C.POINTER(c_void_p), C.POINTER(c_void_p),
                         C.POINTER(c_int), C.POINTER(c_int), c_int, c_int, c_void_p,
                         c_float, c_float, c_float, c_float, c_float, c_void_p, c_int, c_long, c_long, c_void_p,
                         c_void_p, c_int],
        "sc_shadow_rows": [c_void_p, c_void_p, c_void_p, c_long, c_int, c_int, c_void_p],
        "sc_bias_loss": [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int,
                         c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_void_p, c_int, c_int, c_int, c_float, c_float, c_float, c_float,
                         c_float, c_float, c_int, c_void_p, c_void_p, c_int, c_int],
    }
    optional = {
        "sc_topk_select": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                           c_void_p],
        "sc_topk_decode_grad": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_void_p, c_void_p,
                                c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                c_int],
        "sc_topk_sparse_wgrad": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_void_p,
                                 c_int, c_int, c_int, c_int, c_int, c_float, c_int, c_void_p],
        "sc_topk_slot_lists": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                               c_int, c_int, c_void_p],
        "sc_topk_clear": [c_void_p, c_void_p, c_void_p, c_long, c_int, c_int, c_void_p],
        "sc_topk_scatter": [c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_int, c_int, c_int, c_void_p],
        "sc_fista": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                     c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                     c_void_p, c_int],
        "sc_center_rows": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p],
        "sc_gather_rows": [c_void_p, c_void_p, c_void_p, c_long, c_long, c_void_p],
        "sc_gather_rows_perm": [c_void_p, c_long, c_void_p, c_long, c_void_p, c_void_p, c_void_p, c_long, c_long,
                                c_long, c_long, c_long, c_long, c_void_p],
        "sc_gather_rows_blocks": [c_void_p, c_long, c_void_p, c_long, c_long, c_long, c_long, c_long, c_void_p,
                                  c_long, c_void_p],
        "sc_lista_fwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                         c_int, c_void_p],
        "sc_lista_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p],
        "sc_lista_fwd2": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                          c_void_p, c_int, c_int, c_int, c_void_p],
        "sc_lista_bwd2": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                          c_void_p, c_void_p, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                          c_int, c_void_p],
        "sc_res_fwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                       c_void_p],
        "sc_res_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                       c_int, c_int, c_void_p],
        "sc_synth_codes": [c_void_p, c_void_p, c_long, c_int, C.c_ulonglong, C.c_ulonglong, c_void_p],
        "sc_coef_search": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                           c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_float, c_float, c_void_p],
        "sc_fista_adjoint": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                             c_float, c_float, c_int, c_int, c_int, c_int, c_int, c_void_p],
        "sc_fista_adjoint_init": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p],
        "sc_fista_gram": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                          c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p,
                          c_void_p, c_void_p],
        "sc_stream_create_cumask": [c_void_p, c_int, C.POINTER(c_void_p)],
        "sc_stream_destroy": [c_void_p],
        "sc_graph_upload": [c_void_p, c_void_p],
        "sc_step_tail": [c_int, C.POINTER(c_void_p), C.POINTER(c_void_p), C.POINTER(c_void_p),
                         C.POINTER(c_void_p), C.POINTER(c_void_p), C.POINTER(c_void_p),
                         C.POINTER(c_int), C.POINTER(c_int), c_int, c_int, c_void_p, c_float, c_float, c_float,
                         c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int,
                         c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float,
                         c_void_p, c_void_p, c_void_p, c_long, c_void_p, c_long, c_void_p, c_void_p, c_long, c_long,
                         c_int, c_long, c_void_p, c_int, c_long, c_void_p, c_void_p],
        "sc_topk_select_bf16": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                                c_void_p, c_long, c_void_p, c_int, c_void_p],
        "sc_topk_tail": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                         c_void_p, c_float, c_float, c_float, c_void_p, c_int, c_void_p, c_int, c_float, c_void_p,
                         c_void_p, c_void_p, c_long, c_void_p, c_long, c_void_p, c_void_p, c_long, c_long, c_void_p],
        "sc_hessian_ema": [c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_void_p],
        "sc_basis_apply": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_int, c_int,
                           c_void_p],
    }
    return sig, optional


def _declare(lib):
    sig, optional = signatures()
    for name, args in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = c_int
    for name, args in optional.items():
        if hasattr(lib, name):
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = c_int
    return _Checked(lib)


class _Checked:
    """The loaded library with arity-checked entry points: ctypes passes surplus arguments
    with default conversions (a Python int becomes a 32-bit C int), so a call with more
    arguments than the declared signature would silently truncate pointers.  Refuse instead."""

    def __init__(self, lib):
        self._lib = lib
        self._fns = {}

    def __getattr__(self, name):
        fn = self._fns.get(name)
        if fn is None:
            raw = getattr(self._lib, name)
            nargs = len(raw.argtypes) if raw.argtypes is not None else None

            def fn(*args, _raw=raw, _n=nargs, _name=name):
                if _n is not None and len(args) != _n:
                    raise TypeError(f"{_name} takes {_n} arguments, got {len(args)}")
                return _raw(*args)

            self._fns[name] = fn
        return fn


def verify_provenance(path: Path = _LIB_PATH) -> str:
    """Check that the library at ``path`` was built from this tree's kernel sources (the sha256
    ``build.source_hash()`` compiled into it); raises ``KernelError`` otherwise.  Returns the hash."""
    from . import build as _build

    want = _build.source_hash()
    have = _build.embedded_hash(path)
    if have != want:
        raise KernelError(f"{path.name} was built from different kernel sources (library {have[:12] or 'untagged'}, "
                          f"tree {want[:12]}): rebuild with `python -m sparse_coding__amd.ops.build`")
    return want


def lib():
    """Return the loaded kernel library, building it in-tree if it is missing.  A library built
    from other sources than this tree's is refused (``verify_provenance``), never loaded."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not _LIB_PATH.exists():
            if os.environ.get("SC_NO_AUTOBUILD"):
                raise KernelError(f"{_LIB_PATH} missing and SC_NO_AUTOBUILD is set")
            from . import build as _build

            _build.build(verbose=False)
        want = verify_provenance(_LIB_PATH)
        lib_ = C.CDLL(str(_LIB_PATH), mode=C.RTLD_GLOBAL)
        lib_.sc_source_hash.restype = C.c_char_p
        got = lib_.sc_source_hash().decode()
        if got != want:  # (the bytes check above and the loaded symbol must agree)
            raise KernelError(f"loaded {_LIB_PATH.name} reports source hash {got[:12]}, tree is {want[:12]}")
        _lib = _declare(lib_)
        return _lib


def available() -> bool:
    """True when the fused HIP path can run (GPU present and library loadable)."""
    if not torch.cuda.is_available():
        return False
    try:
        lib()
        return True
    except Exception:  # pragma: no cover - reported by callers that require it
        return False


_DEBUG_SYNC = os.environ.get("SC_DEBUG_SYNC", "0") not in ("", "0")


def set_debug_sync(on: bool):
    """Synchronise after every kernel launch and surface asynchronous faults at the
    launch that caused them (``utils.debug.debug_mode``; env ``SC_DEBUG_SYNC=1``)."""
    global _DEBUG_SYNC
    _DEBUG_SYNC = bool(on)


def check(rc: int, what: str):
    if rc != 0:
        raise KernelError(f"{what} failed with code {rc}")
    if _DEBUG_SYNC and torch.cuda.is_available() and not torch.cuda.is_current_stream_capturing():
        try:
            torch.cuda.current_stream().synchronize()
        except RuntimeError as e:  # a fault inside the kernel just launched
            raise KernelError(f"{what} faulted: {e}") from e


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def cu_mask_stream(cus, n_cus: int = 256, device=None):
    """A torch stream whose kernels run only on compute units ``cus`` (iterable of CU ids),
    created with hipExtStreamCreateWithCUMask (csrc/streams.hip)."""
    words = (C.c_uint32 * ((n_cus + 31) // 32))()
    for c in cus:
        words[c // 32] |= 1 << (c % 32)
    out = c_void_p()
    rc = lib().sc_stream_create_cumask(C.cast(words, c_void_p), len(words), C.byref(out))
    check(rc, "sc_stream_create_cumask")
    return torch.cuda.ExternalStream(out.value, device=device)


def stream_handle(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def upload_graph(g: "torch.cuda.CUDAGraph", device=None):
    """hipGraphUpload a captured graph on the current stream, so its first ``replay()`` does not
    pay the upload (csrc/streams.hip)."""
    rc = lib().sc_graph_upload(g.raw_cuda_graph_exec(), stream_handle(device))
    check(rc, "sc_graph_upload")
