"""Checkpoint-compatibility alias of reference ``autoencoders/nmf.py``.

Pickled ``learned_dicts.pt`` files name their classes by this module path; the
classes here are thin subclasses of the native ones in ``sparse_coding__amd.baselines.ica``
so old checkpoints load into the native implementation and new checkpoints can be
written with the reference layout (``sparse_coding__amd.utils.checkpoint``)."""

from sparse_coding__amd.baselines.ica import (  # noqa: F401
    NMFEncoder as _NMFEncoder,
)


class NMFEncoder(_NMFEncoder):
    __doc__ = _NMFEncoder.__doc__
