"""BERT pretraining samples (reference ``megatron/data/bert_dataset.py``).

Sample ``idx`` = sentences ``[start, end)`` of the shuffled sentence map,
split into segments A/B (sentence-order head) or used whole, truncated to the
map's target length, wrapped in ``[CLS] .. [SEP]`` and whole-word masked.
The per-sample RNG is ``RandomState((seed + idx) % 2**32)`` as in the
reference, so samples are identical across frameworks.
"""
import numpy as np
import torch

from .. import global_vars
from .dataset_utils import get_samples_mapping
from .masking import (create_masked_lm_predictions, create_tokens_and_tokentypes,
                      get_a_and_b_segments, pad_and_convert_to_numpy, truncate_segments)


class BertDataset(torch.utils.data.Dataset):
    def __init__(self, name, indexed_dataset, data_prefix, num_epochs, max_num_samples,
                 masked_lm_prob, max_seq_length, short_seq_prob, seed, binary_head):
        self.name = name
        self.seed = seed
        self.masked_lm_prob = masked_lm_prob
        self.max_seq_length = max_seq_length
        self.binary_head = binary_head
        self.indexed_dataset = indexed_dataset
        # 3 special tokens: [CLS] A [SEP] B [SEP]
        self.samples_mapping = get_samples_mapping(indexed_dataset, data_prefix, num_epochs,
                                                   max_num_samples, max_seq_length - 3,
                                                   short_seq_prob, seed, name, binary_head)
        tok = global_vars.get_tokenizer()
        self.vocab_id_list = list(tok.inv_vocab.keys())
        self.vocab_id_to_token_dict = tok.inv_vocab
        self.cls_id, self.sep_id, self.mask_id, self.pad_id = tok.cls, tok.sep, tok.mask, tok.pad

    def __len__(self):
        return self.samples_mapping.shape[0]

    def __getitem__(self, idx):
        start, end, seq_length = (int(v) for v in self.samples_mapping[idx])
        sample = [self.indexed_dataset[i] for i in range(start, end)]
        np_rng = np.random.RandomState(seed=((self.seed + idx) % 2 ** 32))
        return build_training_sample(sample, seq_length, self.max_seq_length,
                                     self.vocab_id_list, self.vocab_id_to_token_dict,
                                     self.cls_id, self.sep_id, self.mask_id, self.pad_id,
                                     self.masked_lm_prob, np_rng, self.binary_head)


def build_training_sample(sample, target_seq_length, max_seq_length, vocab_id_list,
                          vocab_id_to_token_dict, cls_id, sep_id, mask_id, pad_id,
                          masked_lm_prob, np_rng, binary_head):
    """One BERT sample dict: text, types, labels, is_random, loss_mask,
    padding_mask, truncated."""
    if binary_head and len(sample) < 2:
        raise AssertionError("the sentence-order head needs >= 2 sentences per sample")
    if target_seq_length > max_seq_length:
        raise AssertionError("target length exceeds max_seq_length")
    if binary_head:
        tokens_a, tokens_b, is_next_random = get_a_and_b_segments(sample, np_rng)
    else:
        tokens_a = [t for sent in sample for t in sent]
        tokens_b, is_next_random = [], False
    truncated = truncate_segments(tokens_a, tokens_b, len(tokens_a), len(tokens_b),
                                  target_seq_length, np_rng)
    tokens, tokentypes = create_tokens_and_tokentypes(tokens_a, tokens_b, cls_id, sep_id)
    tokens, positions, labels, _, _ = create_masked_lm_predictions(
        tokens, vocab_id_list, vocab_id_to_token_dict, masked_lm_prob, cls_id, sep_id, mask_id,
        masked_lm_prob * target_seq_length, np_rng)
    text, types, labels_np, padding_mask, loss_mask = pad_and_convert_to_numpy(
        tokens, tokentypes, positions, labels, pad_id, max_seq_length)
    return {"text": text, "types": types, "labels": labels_np,
            "is_random": int(is_next_random), "loss_mask": loss_mask,
            "padding_mask": padding_mask, "truncated": int(truncated)}
