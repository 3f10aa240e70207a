"""Dataset split / blend utilities (reference ``megatron/data/dataset_utils.py``).

Split/blend helpers shared by every dataset, plus the sentence-level (BERT /
T5 / ICT) dataset builder and sample-map cache; the masking primitives live in
``masking.py`` and are re-exported here under the reference's names.
"""
import math
import time

import numpy as np

from ..utils.misc import print_rank_0
from . import indexed_dataset


def get_datasets_weights_and_num_samples(data_prefix, train_valid_test_num_samples):
    """``[w1, p1, w2, p2, ...]`` -> (prefixes, normalised weights, per-dataset samples).

    Per-dataset sample counts are over-provisioned by 0.5% so that the greedy
    blend never runs a component dry (reference :44-79).
    """
    if len(data_prefix) % 2:
        raise ValueError("--data_path with several corpora must be 'weight prefix' pairs")
    weights = np.array([float(w) for w in data_prefix[0::2]], dtype=np.float64)
    prefixes = [p.strip() for p in data_prefix[1::2]]
    if weights.sum() <= 0:
        raise ValueError("blend weights must sum to a positive value")
    weights = (weights / weights.sum()).tolist()
    if isinstance(train_valid_test_num_samples, (list, tuple)):
        per = [[int(math.ceil(n * w * 1.005)) for n in train_valid_test_num_samples]
               for w in weights]
    else:
        per = [int(math.ceil(train_valid_test_num_samples * w * 1.005)) for w in weights]
    return prefixes, weights, per


def get_train_valid_test_split_(splits_string, size):
    """Document boundaries ``[0, a, b, size]`` of a "train,valid,test" split (reference :616-640).

    Fractions are normalised, each split rounds independently and the rounding
    excess is taken from every boundary after the first.
    """
    sep = "," if "," in splits_string else ("/" if "/" in splits_string else None)
    parts = [float(s) for s in splits_string.split(sep)] if sep else [float(splits_string)]
    parts = (parts + [0.0, 0.0])[:3]
    total = sum(parts)
    if total <= 0:
        raise ValueError(f"invalid --split {splits_string!r}")
    bounds = [0]
    for p in parts:
        bounds.append(bounds[-1] + int(round(p / total * float(size))))
    excess = bounds[-1] - size
    bounds = [bounds[0]] + [b - excess for b in bounds[1:]]
    assert len(bounds) == 4 and bounds[-1] == size
    return bounds


def get_indexed_dataset_(data_prefix, data_impl, skip_warmup):
    print_rank_0(" > building dataset index ...")
    t0 = time.time()
    ds = indexed_dataset.make_dataset(data_prefix, data_impl, skip_warmup)
    if ds is None:
        raise FileNotFoundError(f"could not open indexed dataset {data_prefix!r}")
    print_rank_0(f" > finished creating indexed dataset in {time.time() - t0:4f} seconds")
    print_rank_0(f"    number of documents: {ds.sizes.shape[0]}")
    print_rank_0(f"    number of tokens: {int(np.asarray(ds.sizes, dtype=np.int64).sum())}")
    return ds


def compile_helper():
    """The reference compiled ``helpers.cpp`` at run time with ``make``; here the
    helper is built ahead of time by ``python -m epfl_megatron_amd.build``."""
    from ..build import build_data_helpers
    build_data_helpers()


# ---- sentence-level datasets (BERT / T5 / ICT) -------------------------------
# Re-exported for the reference's import paths (megatron.data.dataset_utils.*).
from .masking import (get_a_and_b_segments, truncate_segments,  # noqa: E402,F401
                      create_tokens_and_tokentypes, create_masked_lm_predictions,
                      pad_and_convert_to_numpy, is_start_piece, MaskedLmInstance)

DSET_TYPE_BERT = "standard_bert"
DSET_TYPE_ICT = "ict"
DSET_TYPE_T5 = "t5"
DSET_TYPES = [DSET_TYPE_BERT, DSET_TYPE_ICT, DSET_TYPE_T5]


def _mapping_filename(data_prefix, name, num_epochs, max_num_samples, max_seq_length,
                      short_seq_prob, seed, extra=""):
    # Same name as the reference (:660-671) so cached maps are found by both.
    f = f"{data_prefix}_{name}_indexmap"
    if num_epochs != np.iinfo(np.int32).max - 1:
        f += f"_{num_epochs}ep"
    if max_num_samples != np.iinfo(np.int64).max - 1:
        f += f"_{max_num_samples}mns"
    f += f"_{max_seq_length}msl"
    if short_seq_prob is not None:
        f += f"_{short_seq_prob:0.2f}ssp"
    f += extra + f"_{seed}s.npy"
    return f


def _cached_mapping(filename, build, what):
    """Build on global rank 0 (plain .npy, never pickled), barrier, then every
    rank memory-maps the file read-only."""
    import os
    from .gpt_dataset import _barrier, _is_rank0
    if _is_rank0() and not os.path.isfile(filename):
        print(f" > WARNING: could not find index map file {filename}, building the "
              f"{what} indices on rank 0 ...", flush=True)
        t0 = time.time()
        arr = build()
        np.save(filename, arr, allow_pickle=False)
        print_rank_0(f" > saved the index mapping in {filename} "
                     f"({time.time() - t0:4f} s)")
    _barrier()
    arr = np.load(filename, allow_pickle=False, mmap_mode="r")
    print_rank_0(f"    total number of samples: {arr.shape[0]}")
    return arr


def get_samples_mapping(indexed_dataset, data_prefix, num_epochs, max_num_samples,
                        max_seq_length, short_seq_prob, seed, name, binary_head):
    """``[n, 3]`` (first sentence, end sentence, target length) sample map
    (reference :643-729, built by the native ``helpers.build_mapping``)."""
    from . import helpers
    if not num_epochs:
        if not max_num_samples:
            raise ValueError("Need to specify either max_num_samples or num_epochs")
        num_epochs = np.iinfo(np.int32).max - 1
    if not max_num_samples:
        max_num_samples = np.iinfo(np.int64).max - 1
    fname = _mapping_filename(data_prefix, name, num_epochs, max_num_samples, max_seq_length,
                              short_seq_prob, seed)
    return _cached_mapping(fname, lambda: helpers.build_mapping(
        indexed_dataset.doc_idx, indexed_dataset.sizes, num_epochs, max_num_samples,
        max_seq_length, short_seq_prob, seed, _rank0_verbose(), 2 if binary_head else 1),
        "samples")


def _rank0_verbose():
    from .gpt_dataset import _is_rank0
    return _is_rank0()


def build_train_valid_test_datasets(data_prefix, data_impl, splits_string,
                                    train_valid_test_num_samples, max_seq_length,
                                    masked_lm_prob, short_seq_prob, seed, skip_warmup,
                                    binary_head=False, max_seq_length_dec=None,
                                    dataset_type=DSET_TYPE_BERT):
    """BERT / T5 / ICT train-valid-test datasets over sentence-split corpora
    (``preprocess_data.py --split_sentences``), optionally blended (reference
    :421-600)."""
    from .blendable_dataset import BlendableDataset
    if dataset_type not in DSET_TYPES:
        raise ValueError(f"Invalid dataset_type: {dataset_type}")
    if len(data_prefix) == 1:
        return _build_sentence_datasets(data_prefix[0], data_impl, splits_string,
                                        train_valid_test_num_samples, max_seq_length,
                                        masked_lm_prob, short_seq_prob, seed, skip_warmup,
                                        binary_head, max_seq_length_dec, dataset_type)
    prefixes, weights, per_ds = get_datasets_weights_and_num_samples(
        data_prefix, train_valid_test_num_samples)
    parts = [[], [], []]
    for prefix, n in zip(prefixes, per_ds):
        for split, ds in enumerate(_build_sentence_datasets(
                prefix, data_impl, splits_string, n, max_seq_length, masked_lm_prob,
                short_seq_prob, seed, skip_warmup, binary_head, max_seq_length_dec,
                dataset_type)):
            if ds is not None:
                parts[split].append(ds)
    return tuple(BlendableDataset(p, weights) if p else None for p in parts)


def _build_sentence_datasets(data_prefix, data_impl, splits_string, num_samples,
                             max_seq_length, masked_lm_prob, short_seq_prob, seed, skip_warmup,
                             binary_head, max_seq_length_dec, dataset_type):
    ds = get_indexed_dataset_(data_prefix, data_impl, skip_warmup)
    if ds.sizes.shape[0] != ds.doc_idx[-1]:
        raise AssertionError("corpus is not sentence-split (doc_idx[-1] != #sentences)")
    titles = None
    if dataset_type == DSET_TYPE_ICT:
        from .. import global_vars
        titles = get_indexed_dataset_(global_vars.get_args().titles_data_path, data_impl,
                                      skip_warmup)
    ndocs = ds.doc_idx.shape[0] - 1
    bounds = get_train_valid_test_split_(splits_string, ndocs)
    full_doc_idx = ds.get_doc_idx()
    out = []
    for i, name in enumerate(("train", "valid", "test")):
        lo, hi = bounds[i], bounds[i + 1]
        print_rank_0(f"    {name}:\n     document indices in [{lo}, {hi}) total of "
                     f"{hi - lo} documents")
        if hi <= lo:
            out.append(None)
            continue
        # the dataset sees only its split's documents (doc_idx view), as in the reference
        ds.set_doc_idx(full_doc_idx[lo:hi + 1])
        kw = dict(name=name, data_prefix=data_prefix, num_epochs=None,
                  max_num_samples=num_samples[i], max_seq_length=max_seq_length, seed=seed)
        try:
            if dataset_type == DSET_TYPE_ICT:
                from .. import global_vars
                from .ict_dataset import ICTDataset
                a = global_vars.get_args()
                out.append(ICTDataset(block_dataset=ds, title_dataset=titles,
                                      query_in_block_prob=a.query_in_block_prob,
                                      use_one_sent_docs=a.use_one_sent_docs,
                                      binary_head=binary_head, **kw))
            elif dataset_type == DSET_TYPE_T5:
                from .t5_dataset import T5Dataset
                out.append(T5Dataset(indexed_dataset=ds, masked_lm_prob=masked_lm_prob,
                                     max_seq_length_dec=max_seq_length_dec,
                                     short_seq_prob=short_seq_prob, **kw))
            else:
                from .bert_dataset import BertDataset
                out.append(BertDataset(indexed_dataset=ds, masked_lm_prob=masked_lm_prob,
                                       short_seq_prob=short_seq_prob, binary_head=binary_head,
                                       **kw))
        finally:
            ds.set_doc_idx(full_doc_idx)
    return tuple(out)
