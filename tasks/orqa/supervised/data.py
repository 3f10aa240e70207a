"""Supervised retriever data: DPR-format NQ JSON (reference
``tasks/orqa/supervised/data.py``).

Each record has ``question``, ``answers``, ``positive_ctxs`` (the first is
used), ``negative_ctxs`` and ``hard_negative_ctxs`` (``{"title", "text"}``).
Queries are ``[CLS] q [SEP]``, contexts ``[CLS] title [SEP] text [SEP]``.
Validation samples carry ``val_av_rank_other_neg`` + ``val_av_rank_hard_neg``
negatives; with ``--train_with_neg`` training samples carry
``train_hard_neg`` shuffled hard negatives topped up with plain negatives.
"""
import json
import random

import numpy as np
from torch.utils.data import Dataset

from epfl_megatron_amd import get_args, print_rank_0
from epfl_megatron_amd.data.ict_dataset import make_attention_mask
from epfl_megatron_amd.data.orqa_wiki_dataset import build_tokens_types_paddings_from_ids


def _encode_context(ctx, tokenizer, max_seq_length):
    ids = tokenizer.tokenize(ctx["title"]) + [tokenizer.sep] + tokenizer.tokenize(ctx["text"])
    return build_tokens_types_paddings_from_ids(ids, max_seq_length, tokenizer.cls,
                                                tokenizer.sep, tokenizer.pad)


def build_token_types_from_context_list(ctx_list, tokenizer, max_seq_length):
    enc = [_encode_context(c, tokenizer, max_seq_length) for c in ctx_list]
    return [e[0] for e in enc], [e[1] for e in enc]


def build_sample(query_ids, query_types, query_pad_mask, ctx_ids, ctx_types, ctx_pad_mask,
                 answers, neg_ctx_id_list=None, neg_ctx_types_list=None, include_neg=False):
    q = np.asarray(query_ids, dtype=np.int64)
    c = np.asarray(ctx_ids, dtype=np.int64)
    s = {"query": q, "query_mask": make_attention_mask(q, q),
         "query_types": np.asarray(query_types, dtype=np.int64),
         "query_pad_mask": query_pad_mask, "context": c, "context_mask": make_attention_mask(c, c),
         "context_types": np.asarray(ctx_types, dtype=np.int64),
         "context_pad_mask": ctx_pad_mask, "reference": answers}
    if include_neg:
        n = np.asarray(neg_ctx_id_list, dtype=np.int64).reshape(-1, len(q))
        s["neg_context"] = n
        s["neg_context_types"] = np.asarray(neg_ctx_types_list, dtype=np.int64).reshape(n.shape)
        s["neg_context_mask"] = np.stack([make_attention_mask(x, x) for x in n]) if len(n) \
            else np.zeros((0, len(q), len(q)), np.int64)
    return s


def normalize_question(question):
    return question[:-1] if question.endswith("?") else question


class NQSupervisedDataset(Dataset):
    def __init__(self, name, datapaths, tokenizer, max_seq_length, evaluate=False):
        args = get_args()
        self.task_name, self.dataset_name = "natural_questions_ret", name
        self.tokenizer, self.max_seq_length, self.evaluate = tokenizer, max_seq_length, evaluate
        self.val_av_rank_hard_neg = args.val_av_rank_hard_neg
        self.val_av_rank_other_neg = args.val_av_rank_other_neg
        self.train_with_neg, self.train_hard_neg = args.train_with_neg, args.train_hard_neg
        print_rank_0(f" > building {self.task_name} dataset for {name}:")
        self.samples = []
        for p in ([datapaths] if isinstance(datapaths, str) else datapaths):
            self.samples.extend(self.process_samples_from_single_path(p))
        if args.sample_rate < 1:
            self.samples = random.sample(self.samples, int(len(self.samples) * args.sample_rate))
        print_rank_0(f"  >> total number of samples: {len(self.samples)}")

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, idx):
        s = self.samples[idx]
        tok, n = self.tokenizer, self.max_seq_length
        q_ids, q_types, q_pad = build_tokens_types_paddings_from_ids(
            tok.tokenize(s["question"]), n, tok.cls, tok.sep, tok.pad)
        c_ids, c_types, c_pad = _encode_context(s["pos_context"], tok, n)
        neg = None
        if self.evaluate:
            neg = s["negative_context"][:self.val_av_rank_other_neg] + \
                s["hard_negative_context"][:self.val_av_rank_hard_neg]
        elif self.train_with_neg:
            hard, other = list(s["hard_negative_context"]), list(s["negative_context"])
            random.shuffle(hard)
            random.shuffle(other)
            neg = hard[:self.train_hard_neg]
            neg += other[:self.train_hard_neg - len(neg)]
        neg_ids, neg_types = build_token_types_from_context_list(neg, tok, n) if neg is not None \
            else (None, None)
        return build_sample(q_ids, q_types, q_pad, c_ids, c_types, c_pad, s["answers"], neg_ids,
                            neg_types, include_neg=neg is not None)

    @staticmethod
    def process_samples_from_single_path(filename):
        print_rank_0(f" > Processing {filename} ...")
        with open(filename, "r", encoding="utf-8") as f:
            data = json.load(f)
        out = [{"question": normalize_question(r["question"]),
                "pos_context": r["positive_ctxs"][0],
                "hard_negative_context": list(r.get("hard_negative_ctxs") or []),
                "negative_context": list(r.get("negative_ctxs") or []),
                "answers": r["answers"]} for r in data]
        print_rank_0(f" >> processed {len(out)} samples.")
        return out
