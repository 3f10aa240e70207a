"""Zero-shot evaluation datasets (reference tasks/zeroshot_gpt/datasets.py).

* WikiText-103 style LM loss: the detokenised text is tokenised once and cut
  into ``seq_length`` windows that advance by ``--overlapping_eval`` tokens;
  only the last ``overlapping_eval`` targets of every window after the first
  are scored, so each token is predicted exactly once with long context.
* LAMBADA: predict the last word; in ``--strict_lambada`` mode the last
  whitespace word is tokenised separately (its tokens are the targets).
"""
import json
import math

import numpy as np
import torch

from epfl_megatron_amd import get_args, get_tokenizer, print_rank_0
from .detokenizer import get_detokenizer


class LMDataset(torch.utils.data.Dataset):

    def __init__(self, tokens, seq_len, pad_idx, num_original_tokens, num_tokenized_tokens,
                 overlapping_eval=None):
        self.tokens = list(tokens)
        self.seq_len = seq_len
        self.pad_idx = pad_idx
        self.stride = max(1, overlapping_eval if overlapping_eval is not None else seq_len)
        self.num_original_tokens = num_original_tokens
        self.num_tokenized_tokens = num_tokenized_tokens
        # window 0 scores targets 1..seq_len; every later window adds `stride`
        rest = max(len(self.tokens) - 1 - seq_len, 0)
        self.total_sequences = 1 + math.ceil(rest / self.stride)

    def __len__(self):
        return self.total_sequences

    def __getitem__(self, idx):
        start = idx * self.stride
        toks = self.tokens[start:start + self.seq_len + 1]
        n = len(toks)
        mask = np.zeros(self.seq_len + 1, dtype=np.int64)
        mask[:n] = 1
        toks = toks + [self.pad_idx] * (self.seq_len + 1 - n)
        mask = mask[1:]
        if self.stride != self.seq_len and idx != 0:
            mask[:-self.stride] = 0
        return {"text": np.array(toks, dtype=np.int64), "pad_mask": mask}


class LambadaDataset(torch.utils.data.Dataset):

    def __init__(self, path, pad_idx, tokenizer, seq_len, strict=False):
        print_rank_0(f"> building lambada dataset from {path} ...")
        self.seq_len, self.pad_idx, self.tokenizer, self.strict = seq_len, pad_idx, tokenizer, strict
        self.tokens, self.labels = [], []
        with open(path) as f:
            for line in f:
                if line.strip():
                    t, l = self._split(json.loads(line)["text"])
                    self.tokens.append(t)
                    self.labels.append(l)

    def _split(self, text):
        if not self.strict:
            toks = self.tokenizer.tokenize(text)
            return toks[:-1], [toks[-1]]
        last = text.split()[-1]
        start = text.rfind(last)
        return self.tokenizer.tokenize(text[:start].strip()), self.tokenizer.tokenize(" " + last)

    def __len__(self):
        return len(self.tokens)

    def __getitem__(self, idx):
        ctx, lab = list(self.tokens[idx]), list(self.labels[idx])
        toks = ctx + lab
        mask = [0] * len(ctx) + [1] * len(lab)
        pad = self.seq_len + 1 - len(toks)
        if pad < 0:  # keep the end (the target) when the context is too long
            toks, mask = toks[-(self.seq_len + 1):], mask[-(self.seq_len + 1):]
            pad = 0
        toks += [self.pad_idx] * pad
        mask += [0] * pad
        return {"text": np.array(toks, dtype=np.int64),
                "pad_mask": np.array(mask[1:], dtype=np.int64)}


def build_dataset(task):
    args = get_args()
    tok = get_tokenizer()
    if not args.valid_data or len(args.valid_data) != 1:
        raise ValueError("--valid_data must name exactly one file")
    path = args.valid_data[0]
    if task == "LAMBADA":
        ds = LambadaDataset(path, tok.eod, tok, args.seq_length, args.strict_lambada)
    elif task == "WIKITEXT103":
        with open(path, "rb") as f:
            text = f.read().decode("utf-8")
        n_orig = len(text.strip().split(" "))
        ids = tok.tokenize(get_detokenizer(path)(text))
        ds = LMDataset(ids, args.seq_length, tok.eod, n_orig, len(ids), args.overlapping_eval)
        print_rank_0(f" > number of original tokens: {n_orig}, number of detokenized tokens: "
                     f"{len(ids)}")
    else:
        raise NotImplementedError(f"dataset for {task} task is not implemented.")
    print_rank_0(f" > found {len(ds)} samples.")
    return ds
