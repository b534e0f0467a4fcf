"""Checkpoint-compatibility alias of reference ``autoencoders/topk_encoder.py``.

Pickled ``learned_dicts.pt`` files name their classes by this module path; the
classes here are thin subclasses of the native ones in ``sparse_coding__amd.models.topk``
so old checkpoints load into the native implementation and new checkpoints can be
written with the reference layout (``sparse_coding__amd.utils.checkpoint``)."""

from sparse_coding__amd.models.topk import (  # noqa: F401
    TopKLearnedDict as _TopKLearnedDict,
    TopKEncoder,
)


class TopKLearnedDict(_TopKLearnedDict):
    __doc__ = _TopKLearnedDict.__doc__
