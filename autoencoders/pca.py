"""Checkpoint-compatibility alias of reference ``autoencoders/pca.py``.

Pickled ``learned_dicts.pt`` files name their classes by this module path; the
classes here are thin subclasses of the native ones in ``sparse_coding__amd.baselines.pca``
so old checkpoints load into the native implementation and new checkpoints can be
written with the reference layout (``sparse_coding__amd.utils.checkpoint``)."""

from sparse_coding__amd.baselines.pca import (  # noqa: F401
    PCAEncoder as _PCAEncoder,
    BatchedPCA,
    BatchedMean,
    calc_pca,
    calc_mean,
)


class PCAEncoder(_PCAEncoder):
    __doc__ = _PCAEncoder.__doc__
