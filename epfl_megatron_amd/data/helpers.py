"""Dataset index helpers (reference ``megatron/data/helpers.cpp`` API names).

Backed by the C++ module ``_helpers`` (built by ``epfl_megatron_amd.build``).
"""
import numpy as np

try:
    from . import _helpers
except ImportError:  # fresh checkout: compile the (CPU-only, g++) module in-tree once
    from ..build import build_data_helpers
    build_data_helpers()
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


def build_mapping(docs, sizes, num_epochs, max_num_samples, max_seq_length, short_seq_prob, seed,
                  verbose, min_num_sent):
    """BERT/T5 sentence samples ``[n, 3]`` = (first sentence, end sentence, target length)."""
    return _helpers.sentence_pair_mapping(np.ascontiguousarray(docs, dtype=np.int64),
                                          np.ascontiguousarray(sizes, dtype=np.int32),
                                          int(num_epochs), int(max_num_samples),
                                          int(max_seq_length), float(short_seq_prob), int(seed),
                                          bool(verbose), int(min_num_sent))


def build_blocks_mapping(docs, sizes, titles_sizes, num_epochs, max_num_samples, max_seq_length,
                         seed, verbose, use_one_sent_blocks):
    """ICT evidence blocks ``[n, 4]`` = (first sentence, end sentence, doc, block id)."""
    return _helpers.block_mapping(np.ascontiguousarray(docs, dtype=np.int64),
                                  np.ascontiguousarray(sizes, dtype=np.int32),
                                  np.ascontiguousarray(titles_sizes, dtype=np.int32),
                                  int(num_epochs), int(max_num_samples), int(max_seq_length),
                                  int(seed), bool(verbose), bool(use_one_sent_blocks))
