"""Wikipedia evidence passages for open-retrieval QA (reference
``megatron/data/orqa_wiki_dataset.py`` and ``biencoder_dataset_utils.py:13-47``).

The evidence file is the DPR ``psgs_w100.tsv`` layout: a header, then
``doc_id <TAB> text <TAB> title``.  A passage is encoded as
``[CLS] title [SEP] text ... [SEP]`` truncated / padded to
``--retriever_seq_length``.
"""
import csv
import random

import numpy as np
import torch
from torch.utils.data import Dataset

from .. import global_vars
from ..parallel import state
from ..parallel import tensor as tensor_parallel
from ..utils.misc import print_rank_0
from .ict_dataset import make_attention_mask
from .samplers import MegatronPretrainingSampler


def get_one_epoch_dataloader(dataset, micro_batch_size=None):
    """One pass over ``dataset`` split across DP ranks, last batch kept
    (indexing jobs must embed every row exactly once)."""
    args = global_vars.get_args()
    sampler = MegatronPretrainingSampler(
        total_samples=len(dataset), consumed_samples=0,
        micro_batch_size=micro_batch_size or args.micro_batch_size,
        data_parallel_rank=state.get_data_parallel_rank(),
        data_parallel_size=state.get_data_parallel_world_size(), drop_last=False)
    return torch.utils.data.DataLoader(dataset, batch_sampler=sampler,
                                       num_workers=args.num_workers,
                                       pin_memory=torch.cuda.is_available())


def get_open_retrieval_wiki_dataset():
    args = global_vars.get_args()
    return OpenRetrievalEvidenceDataset("2018 Wikipedia from DPR codebase", "evidence",
                                        args.evidence_data_path, global_vars.get_tokenizer(),
                                        args.retriever_seq_length)


def get_open_retrieval_batch(data_iterator):
    keys = ["row_id", "context", "context_mask", "context_types", "context_pad_mask"]
    data = None if data_iterator is None else next(data_iterator)
    b = tensor_parallel.broadcast_data(keys, data, torch.int64)
    return (b["row_id"].long(), b["context"].long(), b["context_mask"] < 0.5,
            b["context_types"].long(), b["context_pad_mask"].long())


def build_tokens_types_paddings_from_ids(text_ids, max_seq_length, cls_id, sep_id, pad_id):
    """``[CLS] text [SEP]`` (text cut to ``max_seq_length-2``), padded with ``pad_id``.
    Returns ids, types and the padding mask (1 on real tokens)."""
    ids = [cls_id, *text_ids][:max_seq_length - 1] + [sep_id]
    n = len(ids)
    pad = max_seq_length - n
    ids += [pad_id] * pad
    types = [0] * n + [pad_id] * pad
    return ids, types, np.array([1] * n + [0] * pad, dtype=np.int64)


def build_tokens_types_paddings_from_text(row, tokenizer, max_seq_length):
    ids = tokenizer.tokenize(row["title"]) + [tokenizer.sep] + tokenizer.tokenize(row["text"])
    return build_tokens_types_paddings_from_ids(ids, max_seq_length, tokenizer.cls,
                                                tokenizer.sep, tokenizer.pad)


def build_sample(row_id, context_ids, context_types, context_pad_mask):
    ids = np.asarray(context_ids, dtype=np.int64)
    return {"row_id": row_id, "context": ids, "context_mask": make_attention_mask(ids, ids),
            "context_types": np.asarray(context_types, dtype=np.int64),
            "context_pad_mask": context_pad_mask}


class OpenRetrievalEvidenceDataset(Dataset):
    def __init__(self, task_name, dataset_name, datapath, tokenizer, max_seq_length):
        self.task_name, self.dataset_name = task_name, dataset_name
        self.tokenizer, self.max_seq_length = tokenizer, max_seq_length
        print_rank_0(f" > building {task_name} dataset for {dataset_name}:")
        self.samples, self.id2text = self.process_samples_from_single_path(datapath)
        rate = getattr(global_vars.get_args(), "sample_rate", 1.0)
        if rate < 1:
            self.samples = random.sample(self.samples, int(len(self.samples) * rate))
        print_rank_0(f"  >> total number of samples: {len(self.samples)}")

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, idx):
        row = self.samples[idx]
        ids, types, pad = build_tokens_types_paddings_from_text(row, self.tokenizer,
                                                                self.max_seq_length)
        return build_sample(row["doc_id"], ids, types, pad)

    @staticmethod
    def process_samples_from_single_path(filename):
        print_rank_0(f" > Processing {filename} ...")
        rows, id2text = [], {}
        with open(filename, newline="", encoding="utf-8") as f:
            reader = csv.reader(f, delimiter="\t")
            next(reader, None)
            for r in reader:
                doc_id, text, title = int(r[0]), r[1], r[2]
                assert doc_id not in id2text
                rows.append({"doc_id": doc_id, "text": text, "title": title})
                id2text[doc_id] = (text, title)
        print_rank_0(f" >> processed {len(rows)} samples.")
        return rows, id2text
