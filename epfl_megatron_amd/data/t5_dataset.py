"""T5 span-corruption samples (reference ``megatron/data/t5_dataset.py``).

Spans (geometric lengths, <= 10 words) are replaced in the encoder input by
consecutive sentinel tokens; the decoder reads ``<bos> s0 span0 s1 span1 ...``
and predicts ``s0 span0 s1 span1 ... <eos>``.  Per-sample RNG is
``RandomState(seed + idx)`` (no modulo, as the reference).
"""
import collections

import numpy as np
import torch

from .. import global_vars
from .dataset_utils import get_samples_mapping
from .masking import create_masked_lm_predictions


class T5Dataset(torch.utils.data.Dataset):
    def __init__(self, name, indexed_dataset, data_prefix, num_epochs, max_num_samples,
                 masked_lm_prob, max_seq_length, max_seq_length_dec, short_seq_prob, seed):
        self.name = name
        self.seed = seed
        self.masked_lm_prob = masked_lm_prob
        self.max_seq_length = max_seq_length
        self.max_seq_length_dec = max_seq_length_dec
        self.indexed_dataset = indexed_dataset
        self.samples_mapping = get_samples_mapping(indexed_dataset, data_prefix, num_epochs,
                                                   max_num_samples, max_seq_length - 2,
                                                   short_seq_prob, seed, name, False)
        tok = global_vars.get_tokenizer()
        self.vocab_id_list = list(tok.inv_vocab.keys())
        self.vocab_id_to_token_dict = tok.inv_vocab
        self.cls_id, self.sep_id, self.mask_id, self.pad_id = tok.cls, tok.sep, tok.mask, tok.pad
        self.bos_id = tok.bos_token_id
        self.eos_id = tok.eos_token_id
        self.sentinel_tokens = tok.additional_special_tokens_ids
        if not self.sentinel_tokens:
            raise AssertionError("Provide the argument --vocab_extra_ids 100 to the script")

    def __len__(self):
        return self.samples_mapping.shape[0]

    def __getitem__(self, idx):
        start, end, seq_length = (int(v) for v in self.samples_mapping[idx])
        sample = [self.indexed_dataset[i] for i in range(start, end)]
        np_rng = np.random.RandomState(seed=(self.seed + idx))
        return build_training_sample(sample, seq_length, self.max_seq_length,
                                     self.max_seq_length_dec, self.vocab_id_list,
                                     self.vocab_id_to_token_dict, self.cls_id, self.sep_id,
                                     self.mask_id, self.pad_id, self.masked_lm_prob, np_rng,
                                     self.bos_id, self.eos_id, self.sentinel_tokens)


def build_training_sample(sample, target_seq_length, max_seq_length, max_seq_length_dec,
                          vocab_id_list, vocab_id_to_token_dict, cls_id, sep_id, mask_id, pad_id,
                          masked_lm_prob, np_rng, bos_id=None, eos_id=None,
                          sentinel_tokens=None):
    if target_seq_length > max_seq_length:
        raise AssertionError("target length exceeds max_seq_length")
    tokens = [t for sent in sample for t in sent]
    truncated = len(tokens) > target_seq_length
    tokens = tokens[:target_seq_length]
    tokens, positions, labels, _, spans = create_masked_lm_predictions(
        tokens, vocab_id_list, vocab_id_to_token_dict, masked_lm_prob, cls_id, sep_id, mask_id,
        masked_lm_prob * target_seq_length, np_rng, max_ngrams=10, geometric_dist=True,
        masking_style="t5")
    enc, dec_in, labels_np, enc_mask, dec_mask, enc_dec_mask, loss_mask = \
        pad_and_convert_to_numpy(tokens, positions, labels, pad_id, max_seq_length,
                                 max_seq_length_dec, spans, bos_id, eos_id, sentinel_tokens)
    return {"text_enc": enc, "text_dec": dec_in, "labels": labels_np, "loss_mask": loss_mask,
            "truncated": int(truncated), "enc_mask": enc_mask, "dec_mask": dec_mask,
            "enc_dec_mask": enc_dec_mask}


def pad_and_convert_to_numpy(tokens, masked_positions, masked_labels, pad_id, max_seq_length,
                             max_seq_length_dec, masked_spans=None, bos_id=None, eos_id=None,
                             sentinel_tokens=None):
    sentinels = collections.deque(sentinel_tokens)
    enc, dec_in, dec_out = [], [bos_id], []
    cursor = 0
    for span in masked_spans:
        flag = sentinels.popleft()
        dec_in += [flag] + list(span.label)
        dec_out += [flag] + list(span.label)
        enc += list(tokens[cursor:span.index[0]]) + [flag]
        cursor = span.index[-1] + 1
    dec_out.append(eos_id)
    enc += list(tokens[cursor:])
    pad = max_seq_length - len(enc)
    pad_dec = max_seq_length_dec - len(dec_in)
    if pad < 0 or pad_dec < 0 or len(masked_positions) != len(masked_labels):
        raise AssertionError("sample does not fit max_seq_length / max_seq_length_dec")
    tokens_enc = np.array(enc + [pad_id] * pad, dtype=np.int64)
    tokens_dec_in = np.array(dec_in + [pad_id] * pad_dec, dtype=np.int64)
    enc_mask = make_attention_mask(tokens_enc, tokens_enc)
    enc_dec_mask = make_attention_mask(tokens_dec_in, tokens_enc)
    dec_mask = make_attention_mask(tokens_dec_in, tokens_dec_in) * make_history_mask(tokens_dec_in)
    labels = np.array(dec_out + [-1] * pad_dec, dtype=np.int64)
    loss_mask = np.array([1] * len(dec_in) + [0] * pad_dec, dtype=np.int64)
    return tokens_enc, tokens_dec_in, labels, enc_mask, dec_mask, enc_dec_mask, loss_mask


def make_attention_mask(source_block, target_block):
    """int64 ``[len(source), len(target)]``: 1 where both tokens are non-pad (id >= 1)."""
    return ((target_block[None, :] >= 1) * (source_block[:, None] >= 1)).astype(np.int64)


def make_attention_mask_3d(source_block, target_block):
    return (target_block[:, None, :] >= 1) * (source_block[:, :, None] >= 1)


def make_history_mask(block):
    n = block.shape[0]
    ar = np.arange(n)
    return (ar[None, :] <= ar[:, None]).astype(np.int64)


def make_history_mask_3d(block):
    b, n = block.shape
    ar = torch.arange(n, device=block.device)
    return (ar[None, :] <= ar[:, None])[None].expand(b, n, n)
