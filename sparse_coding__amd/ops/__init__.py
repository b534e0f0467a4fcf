"""gfx950 HIP kernels (C ABI, ctypes-bound) and their host-side wrappers."""

from ._lib import KernelError, available, lib  # noqa: F401
