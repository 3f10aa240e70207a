"""Vocab-parallel cross-entropy (implementation lives in ``ops/cross_entropy``)."""
from ...ops.cross_entropy import vocab_parallel_cross_entropy  # noqa: F401
