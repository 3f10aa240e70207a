"""GPT training samples from indexed corpora (reference ``megatron/data/gpt_dataset.py``).

A sample is ``seq_length + 1`` consecutive tokens of the (epoch-repeated,
document-shuffled) corpus; consecutive samples share one boundary token.  The
three index maps are the reference's, bit for bit, so cached
``<prefix>_<name>_indexmap_<N>ns_<S>sl_<seed>s_{doc,sample,shuffle}_idx.npy``
files are interchangeable in both directions:

* ``doc_idx``     int32 — documents of every epoch, shuffled with
  ``np.random.RandomState(seed)``; when the last epoch contributes < 80% of a
  full epoch it is shuffled separately (reference :305-341, :429-442);
* ``sample_idx``  int32 ``[N+1, 2]`` — (position in doc_idx, offset), built by
  the native helper (reference :354-358);
* ``shuffle_idx`` uint32 (int64 when huge) — permutation of the samples,
  again separating the partial last epoch (reference :494-513).

Maps are built on global rank 0, written as plain ``.npy`` (never pickled),
and every rank then maps them read-only.  Sample assembly goes through the
native ``stitch`` of :class:`MMapIndexedDataset`, batched via
``__getitems__`` so a DataLoader fetches a micro-batch in one C++ call.
"""
import os
import time

import numpy as np
import torch

from ..utils.misc import print_rank_0
from .blendable_dataset import BlendableDataset
from .dataset_utils import (get_datasets_weights_and_num_samples, get_train_valid_test_split_,
                            get_indexed_dataset_)
from . import helpers


def build_train_valid_test_datasets(data_prefix, data_impl, splits_string,
                                    train_valid_test_num_samples, seq_length, seed, skip_warmup,
                                    train_data_prefix=None, valid_data_prefix=None,
                                    test_data_prefix=None):
    """``--data_path`` (one corpus or a weighted blend, split by ``--split``) or
    separate ``--{train,valid,test}_data_path`` lists (reference :20-95)."""
    if data_prefix:
        if len(data_prefix) == 1:
            return _build_train_valid_test_datasets(data_prefix[0], data_impl, splits_string,
                                                    train_valid_test_num_samples, seq_length,
                                                    seed, skip_warmup)
        prefixes, weights, per_ds = get_datasets_weights_and_num_samples(
            data_prefix, train_valid_test_num_samples)
        parts = [[], [], []]
        for prefix, n in zip(prefixes, per_ds):
            for split, ds in enumerate(_build_train_valid_test_datasets(
                    prefix, data_impl, splits_string, n, seq_length, seed, skip_warmup)):
                if ds is not None:
                    parts[split].append(ds)
        # NB: like the reference, the weights of the corpora that produced a
        # split are used (all corpora produce every non-empty split).
        return tuple(BlendableDataset(p, weights) if p else None for p in parts)
    print_rank_0("Separate data paths provided for train, valid & test. "
                 "Split string will be ignored.")
    out = []
    for name, prefix, n, warm in (("train", train_data_prefix, train_valid_test_num_samples[0],
                                   skip_warmup),
                                  ("valid", valid_data_prefix, train_valid_test_num_samples[1],
                                   False),
                                  ("test", test_data_prefix, train_valid_test_num_samples[2],
                                   False)):
        out.append(None if prefix is None else
                   _build_dataset(name, prefix, data_impl, n, seq_length, seed, warm))
    return tuple(out)


def _build_dataset(name, data_prefix, data_impl, num_samples, seq_length, seed, skip_warmup):
    if len(data_prefix) == 1:
        return _whole_corpus(name, data_prefix[0], data_impl, num_samples, seq_length, seed,
                             skip_warmup)
    prefixes, weights, per_ds = get_datasets_weights_and_num_samples(data_prefix, num_samples)
    dss = [_whole_corpus(name, p, data_impl, n, seq_length, seed, skip_warmup)
           for p, n in zip(prefixes, per_ds)]
    dss = [d for d in dss if d is not None]
    return BlendableDataset(dss, weights) if dss else None


def _whole_corpus(name, prefix, data_impl, num_samples, seq_length, seed, skip_warmup):
    ds = get_indexed_dataset_(prefix, data_impl, skip_warmup)
    n = ds.sizes.shape[0]
    print_rank_0(f"    {name}:\n     document indices in [0, {n}) total of {n} documents")
    return GPTDataset(name, prefix, np.arange(n, dtype=np.int32), ds, num_samples, seq_length,
                      seed)


def _build_train_valid_test_datasets(data_prefix, data_impl, splits_string,
                                     train_valid_test_num_samples, seq_length, seed, skip_warmup):
    ds = get_indexed_dataset_(data_prefix, data_impl, skip_warmup)
    bounds = get_train_valid_test_split_(splits_string, ds.sizes.shape[0])
    print_rank_0(" > dataset split:")
    out = []
    for i, name in enumerate(("train", "valid", "test")):
        lo, hi = bounds[i], bounds[i + 1]
        print_rank_0(f"    {name}:\n     document indices in [{lo}, {hi}) total of "
                     f"{hi - lo} documents")
        out.append(GPTDataset(name, data_prefix, np.arange(lo, hi, dtype=np.int32), ds,
                              train_valid_test_num_samples[i], seq_length, seed)
                   if hi > lo else None)
    return tuple(out)


class GPTDataset(torch.utils.data.Dataset):

    def __init__(self, name, data_prefix, documents, indexed_dataset, num_samples, seq_length,
                 seed):
        self.name = name
        self.indexed_dataset = indexed_dataset
        self.seq_length = seq_length
        documents = np.asarray(documents)
        if documents.size and (documents.min() < 0 or
                               documents.max() >= indexed_dataset.sizes.shape[0]):
            raise IndexError("document ids outside the corpus")
        self.doc_idx, self.sample_idx, self.shuffle_idx = _build_index_mappings(
            name, data_prefix, documents, indexed_dataset.sizes, num_samples, seq_length, seed)
        self._native = hasattr(indexed_dataset, "stitch")

    def __len__(self):
        return self.sample_idx.shape[0] - 1

    def _python_sample(self, s):
        (d0, o0), (d1, o1) = self.sample_idx[s], self.sample_idx[s + 1]
        get = self.indexed_dataset.get
        if d0 == d1:
            return np.asarray(get(int(self.doc_idx[d0]), offset=int(o0), length=int(o1 - o0 + 1)),
                              dtype=np.int64)
        parts = [get(int(self.doc_idx[d0]), offset=int(o0))]
        parts += [get(int(self.doc_idx[d])) for d in range(d0 + 1, d1)]
        parts.append(get(int(self.doc_idx[d1]), length=int(o1 + 1)))
        return np.concatenate(parts).astype(np.int64)

    def samples(self, idxs):
        """int64 ``[len(idxs), seq_length + 1]`` for dataset positions ``idxs``."""
        s = np.asarray(self.shuffle_idx[np.asarray(idxs, dtype=np.int64)], dtype=np.int64)
        if self._native:
            return self.indexed_dataset.stitch(self.doc_idx, self.sample_idx, s, self.seq_length)
        return np.stack([self._python_sample(int(i)) for i in s])

    def __getitem__(self, idx):
        return {"text": self.samples([int(idx)])[0]}

    def __getitems__(self, idxs):
        return [{"text": row} for row in self.samples(idxs)]


def _is_rank0():
    return not torch.distributed.is_initialized() or torch.distributed.get_rank() == 0


def _barrier():
    """Barrier over the ranks that build datasets (TP-rank 0 of every DP x PP
    cell, reference :381-386): all-reduce over the DP then the PP group."""
    if not torch.distributed.is_initialized():
        return
    from ..parallel import state
    if not state.model_parallel_is_initialized():
        torch.distributed.barrier()
        return
    dev = "cpu" if torch.distributed.get_backend() == "gloo" else torch.cuda.current_device()
    t = torch.ones(1, dtype=torch.int64, device=dev)
    torch.distributed.all_reduce(t, group=state.get_data_parallel_group())
    torch.distributed.all_reduce(t, group=state.get_pipeline_model_parallel_group())
    want = torch.distributed.get_world_size() // state.get_tensor_model_parallel_world_size()
    if int(t.item()) != want:
        raise RuntimeError(f"dataset barrier reached by {int(t.item())} of {want} ranks")


def _num_tokens(documents, sizes):
    return int(np.sum(np.asarray(sizes)[documents], dtype=np.int64))


def _num_epochs(tokens_per_epoch, seq_length, num_samples):
    """Smallest epoch count with ``(E*tokens - 1) // seq_length >= num_samples``."""
    epochs = 1
    while (epochs * tokens_per_epoch - 1) // seq_length < num_samples:
        epochs += 1
    return epochs


def _build_doc_idx(documents, num_epochs, np_rng, separate_last_epoch):
    if not separate_last_epoch or num_epochs == 1:
        doc_idx = np.tile(np.asarray(documents, dtype=np.int32), num_epochs)
        np_rng.shuffle(doc_idx)
        return doc_idx
    first = _build_doc_idx(documents, num_epochs - 1, np_rng, False)
    last = _build_doc_idx(documents, 1, np_rng, False)
    return np.concatenate((first, last))


def _build_shuffle_idx(num_samples, total_size, np_rng):
    dtype = np.uint32 if total_size < np.iinfo(np.uint32).max - 1 else np.int64
    first = np.arange(num_samples, dtype=dtype)
    np_rng.shuffle(first)
    if num_samples == total_size:
        return first
    last = np.arange(num_samples, total_size, dtype=dtype)
    np_rng.shuffle(last)
    return np.concatenate((first, last))


def _index_map_prefix(data_prefix, name, num_samples, seq_length, seed):
    return f"{data_prefix}_{name}_indexmap_{num_samples}ns_{seq_length}sl_{seed}s"


def _build_index_mappings(name, data_prefix, documents, sizes, num_samples, seq_length, seed):
    tokens_per_epoch = _num_tokens(documents, sizes)
    if tokens_per_epoch <= 1:
        raise ValueError(f"{data_prefix} ({name}): corpus split has no tokens")
    num_epochs = _num_epochs(tokens_per_epoch, seq_length, num_samples)
    base = _index_map_prefix(data_prefix, name, num_samples, seq_length, seed)
    files = [f"{base}_{k}_idx.npy" for k in ("doc", "sample", "shuffle")]

    if _is_rank0() and not all(os.path.isfile(f) for f in files):
        print_rank_0(" > WARNING: could not find index map files, building the indices on "
                     "rank 0 ...")
        np_rng = np.random.RandomState(seed=seed)
        separate_last_epoch = False
        if num_epochs > 1:
            from_full = ((num_epochs - 1) * tokens_per_epoch - 1) // seq_length
            last_epoch = num_samples - from_full
            per_epoch = (tokens_per_epoch - 1) // seq_length
            assert 0 <= last_epoch < per_epoch + 1
            separate_last_epoch = last_epoch < int(0.80 * per_epoch)
            print(f" > last epoch number of samples ({last_epoch}) is "
                  f"{'smaller' if separate_last_epoch else 'larger'} than 80% of number of "
                  f"samples per epoch ({per_epoch}), setting separate_last_epoch to "
                  f"{separate_last_epoch}", flush=True)
        t0 = time.time()
        doc_idx = _build_doc_idx(documents, num_epochs, np_rng, separate_last_epoch)
        sample_idx = helpers.build_sample_idx(np.asarray(sizes, dtype=np.int32), doc_idx,
                                              seq_length, num_epochs, tokens_per_epoch)
        n_first = from_full if separate_last_epoch else sample_idx.shape[0] - 1
        shuffle_idx = _build_shuffle_idx(n_first, sample_idx.shape[0] - 1, np_rng)
        for f, arr in zip(files, (doc_idx, sample_idx, shuffle_idx)):
            tmp = f + f".tmp{os.getpid()}.npy"
            np.save(tmp, arr, allow_pickle=False)
            os.replace(tmp, f)
        print_rank_0(f" > built and saved index maps in {time.time() - t0:4f} seconds")
    _barrier()
    t0 = time.time()
    doc_idx, sample_idx, shuffle_idx = (np.load(f, allow_pickle=False, mmap_mode="r")
                                        for f in files)
    print_rank_0(f"    loaded indexed file in {time.time() - t0:3.3f} seconds\n"
                 f"    total number of tokens: {tokens_per_epoch}\n"
                 f"    total number of samples: {sample_idx.shape[0]}\n"
                 f"    total number of epochs: {num_epochs}")
    return doc_idx, sample_idx, shuffle_idx
