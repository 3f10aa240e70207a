"""Dataset split / blend utilities (reference ``megatron/data/dataset_utils.py``).

Only the GPT-relevant helpers are here; the BERT/T5 masking helpers live with
the legacy datasets.
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
