"""Evidence-block sample maps for ICT / REALM retrieval pretraining
(reference ``megatron/data/realm_dataset_utils.py``)."""
import numpy as np
import torch

from .dataset_utils import _cached_mapping, _rank0_verbose


class BlockSampleData:
    """(first sentence, end sentence, source document, block id) of one block."""

    def __init__(self, start_idx, end_idx, doc_idx, block_idx):
        self.start_idx = int(start_idx)
        self.end_idx = int(end_idx)
        self.doc_idx = int(doc_idx)
        self.block_idx = int(block_idx)

    def as_array(self):
        return np.array([self.start_idx, self.end_idx, self.doc_idx, self.block_idx],
                        dtype=np.int64)

    def as_tuple(self):
        return self.start_idx, self.end_idx, self.doc_idx, self.block_idx


class BlockSamplesMapping:
    def __init__(self, mapping_array):
        if mapping_array.ndim != 2 or mapping_array.shape[1] != 4:
            raise AssertionError("block mapping must be [n, 4]")
        self.mapping_array = mapping_array

    def __len__(self):
        return self.mapping_array.shape[0]

    def __getitem__(self, idx):
        return BlockSampleData(*self.mapping_array[idx])


def get_block_samples_mapping(block_dataset, title_dataset, data_prefix, num_epochs,
                              max_num_samples, max_seq_length, seed, name,
                              use_one_sent_docs=False):
    """Blocks of whole sentences that fit ``max_seq_length - 3 - len(title)``
    (native ``helpers.build_blocks_mapping``), cached like the reference."""
    from . import helpers
    if not num_epochs:
        if not max_num_samples:
            raise ValueError("Need to specify either max_num_samples or num_epochs")
        num_epochs = np.iinfo(np.int32).max - 1
    if not max_num_samples:
        max_num_samples = np.iinfo(np.int64).max - 1
    f = f"{data_prefix}_{name}_indexmap"
    if num_epochs != np.iinfo(np.int32).max - 1:
        f += f"_{num_epochs}ep"
    if max_num_samples != np.iinfo(np.int64).max - 1:
        f += f"_{max_num_samples}mns"
    f += f"_{max_seq_length}msl_{seed}s" + ("_1sentok" if use_one_sent_docs else "") + ".npy"
    arr = _cached_mapping(f, lambda: helpers.build_blocks_mapping(
        block_dataset.doc_idx, block_dataset.sizes, title_dataset.sizes, num_epochs,
        max_num_samples, max_seq_length - 3, seed, _rank0_verbose(), use_one_sent_docs),
        "block")
    return BlockSamplesMapping(arr)


def get_ict_batch(data_iterator):
    """TP-broadcast ICT batch -> (query tokens, query mask, context tokens,
    context mask, block data); masks become bool ``[b, s, s]``, True = masked.

    (The reference's version names keys the ICT dataset never produces;
    these are the dataset's own keys.)"""
    from ..parallel import tensor as tp
    keys = ["query_tokens", "query_mask", "context_tokens", "context_mask", "block_data"]
    data = next(data_iterator) if data_iterator is not None else None
    b = tp.broadcast_data(keys, data, torch.int64)
    return (b["query_tokens"].long(), b["query_mask"] < 0.5, b["context_tokens"].long(),
            b["context_mask"] < 0.5, b["block_data"].long())


def join_str_list(str_list):
    """Detokenize WordPiece strings ('##' continues the previous word)."""
    out = ""
    for s in str_list:
        out += s[2:] if s.startswith("##") else " " + s
    return out
