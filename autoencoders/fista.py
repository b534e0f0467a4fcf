"""Checkpoint-compatibility alias of reference ``autoencoders/fista.py``.

Pickled ``learned_dicts.pt`` files name their classes by this module path; the
classes here are thin subclasses of the native ones in ``sparse_coding__amd.models.fista``
so old checkpoints load into the native implementation and new checkpoints can be
written with the reference layout (``sparse_coding__amd.utils.checkpoint``)."""

from sparse_coding__amd.models.fista import (  # noqa: F401
    Fista as _Fista,
    FunctionalFista,
)


class Fista(_Fista):
    __doc__ = _Fista.__doc__
