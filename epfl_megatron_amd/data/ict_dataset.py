"""Inverse Cloze Task samples (reference ``megatron/data/ict_dataset.py``).

A pseudo-query is one sentence of an evidence block; with probability
``1 - query_in_block_prob`` it is removed from the block.  Query:
``[CLS] q [SEP]``; context: ``[CLS] title [SEP] block [SEP]``, both padded to
``max_seq_length``.  The sentence choice uses ``random.Random(seed)`` owned by
the dataset (reference behaviour: the draw sequence depends on access order).
"""
import itertools
import random

import numpy as np
from torch.utils.data import Dataset

from .. import global_vars
from .dataset_utils import get_indexed_dataset_
from .realm_dataset_utils import get_block_samples_mapping


def make_attention_mask(source_block, target_block):
    return ((target_block[None, :] >= 1) * (source_block[:, None] >= 1)).astype(np.int64)


def get_ict_dataset(use_titles=True, query_in_block_prob=1):
    """Single-epoch dataset over all blocks (for indexing / evaluation)."""
    args = global_vars.get_args()
    blocks = get_indexed_dataset_(args.data_path[0] if isinstance(args.data_path, list)
                                  else args.data_path, "mmap", True)
    titles = get_indexed_dataset_(args.titles_data_path, "mmap", True)
    return ICTDataset(name="full", block_dataset=blocks, title_dataset=titles,
                      data_prefix=args.data_path[0] if isinstance(args.data_path, list)
                      else args.data_path, num_epochs=1, max_num_samples=None,
                      max_seq_length=args.seq_length, seed=1,
                      query_in_block_prob=query_in_block_prob, use_titles=use_titles,
                      use_one_sent_docs=args.use_one_sent_docs)


class ICTDataset(Dataset):
    def __init__(self, name, block_dataset, title_dataset, data_prefix, num_epochs,
                 max_num_samples, max_seq_length, query_in_block_prob, seed, use_titles=True,
                 use_one_sent_docs=False, binary_head=False):
        self.name = name
        self.seed = seed
        self.max_seq_length = max_seq_length
        self.query_in_block_prob = query_in_block_prob
        self.block_dataset = block_dataset
        self.title_dataset = title_dataset
        self.rng = random.Random(seed)
        self.use_titles = use_titles
        self.use_one_sent_docs = use_one_sent_docs
        self.samples_mapping = get_block_samples_mapping(
            block_dataset, title_dataset, data_prefix, num_epochs, max_num_samples,
            max_seq_length, seed, name, use_one_sent_docs)
        tok = global_vars.get_tokenizer()
        self.vocab_id_list = list(tok.inv_vocab.keys())
        self.vocab_id_to_token_list = tok.inv_vocab
        self.cls_id, self.sep_id, self.mask_id, self.pad_id = tok.cls, tok.sep, tok.mask, tok.pad

    def __len__(self):
        return len(self.samples_mapping)

    def __getitem__(self, idx):
        data = self.samples_mapping[idx]
        start, end, doc, _ = data.as_tuple()
        if self.use_titles:
            title = self.title_dataset[doc]
            reserved = 3 + len(title)
        else:
            title, reserved = None, 2
        block = [self.block_dataset[i] for i in range(start, end)]
        if not (len(block) > 1 or self.use_one_sent_docs or self.query_in_block_prob == 1):
            raise AssertionError("single-sentence block")
        pick = self.rng.randint(0, len(block) - 1)
        if self.rng.random() < self.query_in_block_prob:
            query = block[pick].copy()
        else:
            query = block.pop(pick)
        query = query[:self.max_seq_length - 2]
        block = list(itertools.chain(*block))[:self.max_seq_length - reserved]
        q_tok, q_pad = self.concat_and_pad_tokens(query)
        c_tok, c_pad = self.concat_and_pad_tokens(block, title)
        return {"query_tokens": q_tok, "query_mask": make_attention_mask(q_tok, q_tok),
                "query_pad_mask": q_pad, "context_tokens": c_tok,
                "context_mask": make_attention_mask(c_tok, c_tok), "context_pad_mask": c_pad,
                "block_data": data.as_array()}

    def get_block(self, start_idx, end_idx, doc_idx):
        block = [self.block_dataset[i] for i in range(start_idx, end_idx)]
        title = self.title_dataset[int(doc_idx)]
        block = list(itertools.chain(*block))[:self.max_seq_length - (3 + len(title))]
        return self.concat_and_pad_tokens(block, title)

    def get_null_block(self):
        return self.concat_and_pad_tokens([], [])

    def concat_and_pad_tokens(self, tokens, title=None):
        tokens = list(tokens)
        if title is None:
            tokens = [self.cls_id] + tokens + [self.sep_id]
        else:
            tokens = [self.cls_id] + list(title) + [self.sep_id] + tokens + [self.sep_id]
        if len(tokens) > self.max_seq_length:
            raise AssertionError("block longer than max_seq_length")
        pad = self.max_seq_length - len(tokens)
        return (np.array(tokens + [self.pad_id] * pad),
                np.array([1] * len(tokens) + [0] * pad))
