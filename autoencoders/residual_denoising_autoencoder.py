"""Checkpoint-compatibility alias of reference ``autoencoders/residual_denoising_autoencoder.py``.

Pickled ``learned_dicts.pt`` files name their classes by this module path; the
classes here are thin subclasses of the native ones in ``sparse_coding__amd.models.lista``
so old checkpoints load into the native implementation and new checkpoints can be
written with the reference layout (``sparse_coding__amd.utils.checkpoint``)."""

from sparse_coding__amd.models.lista import (  # noqa: F401
    LISTADenoisingSAE as _LISTADenoisingSAE,
    ResidualDenoisingSAE as _ResidualDenoisingSAE,
    FunctionalLISTADenoisingSAE,
    FunctionalResidualDenoisingSAE,
    LISTALayer,
    ResidualDenoisingLayer,
    shrinkage,
)


class LISTADenoisingSAE(_LISTADenoisingSAE):
    __doc__ = _LISTADenoisingSAE.__doc__


class ResidualDenoisingSAE(_ResidualDenoisingSAE):
    __doc__ = _ResidualDenoisingSAE.__doc__
