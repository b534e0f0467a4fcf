"""Checkpoint-compatibility alias of reference ``autoencoders/direct_coef_search.py``.

Pickled ``learned_dicts.pt`` files name their classes by this module path; the
classes here are thin subclasses of the native ones in ``sparse_coding__amd.models.misc``
so old checkpoints load into the native implementation and new checkpoints can be
written with the reference layout (``sparse_coding__amd.utils.checkpoint``)."""

from sparse_coding__amd.models.misc import (  # noqa: F401
    DirectCoefSearch as _DirectCoefSearch,
    DirectCoefOptimizer,
)


class DirectCoefSearch(_DirectCoefSearch):
    __doc__ = _DirectCoefSearch.__doc__
