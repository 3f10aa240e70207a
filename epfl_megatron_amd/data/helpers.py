"""Dataset index helpers (reference ``megatron/data/helpers.cpp`` API names).

Backed by the C++ module ``_helpers`` (built by ``epfl_megatron_amd.build``).
"""
import numpy as np

from . import _helpers


def build_sample_idx(sizes, doc_idx, seq_length, num_epochs, tokens_per_epoch):
    return _helpers.sample_index(np.ascontiguousarray(sizes, dtype=np.int32),
                                 np.ascontiguousarray(doc_idx, dtype=np.int32),
                                 int(seq_length), int(num_epochs), int(tokens_per_epoch))


def build_blending_indices(dataset_index, dataset_sample_index, weights, num_datasets, size,
                           verbose):
    """Fills ``dataset_index`` (uint8) / ``dataset_sample_index`` (int64) in place."""
    which, within = _helpers.blend_indices(np.ascontiguousarray(weights, dtype=np.float64),
                                           int(size), bool(verbose))
    dataset_index[:] = which
    dataset_sample_index[:] = within


def stitch_samples(tokens, pointers, sizes, doc_idx, sample_idx, samples, seq_length):
    """int64 ``[len(samples), seq_length + 1]`` GPT samples gathered natively."""
    return _helpers.stitch_samples(tokens, np.ascontiguousarray(pointers, dtype=np.int64),
                                   np.ascontiguousarray(sizes, dtype=np.int32),
                                   np.ascontiguousarray(doc_idx, dtype=np.int32),
                                   np.ascontiguousarray(sample_idx, dtype=np.int32),
                                   np.ascontiguousarray(np.atleast_1d(samples), dtype=np.int64),
                                   int(seq_length))
