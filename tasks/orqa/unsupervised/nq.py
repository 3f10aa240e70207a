"""Google Natural Questions retrieval-eval set (reference
``tasks/orqa/unsupervised/nq.py``): TSV rows ``question <TAB> [answers]``,
encoded as ``[CLS] question [SEP]`` padded to ``--retriever_seq_length``.

The answer list is parsed with ``ast.literal_eval`` (the reference calls
``eval`` on file contents)."""
import ast
import csv

import numpy as np
import torch
from torch.utils.data import BatchSampler, DataLoader, Dataset, SequentialSampler

from epfl_megatron_amd import get_args, get_tokenizer, print_rank_0
from epfl_megatron_amd.data.ict_dataset import make_attention_mask
from epfl_megatron_amd.data.orqa_wiki_dataset import build_tokens_types_paddings_from_ids


def get_nq_dataset(qa_data, split):
    return NQDataset(f"Google NQ {split} Split", "Google Natural Questions", qa_data,
                     get_tokenizer(), get_args().retriever_seq_length)


def _device():
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
        else torch.device("cpu")


def process_nq_batch(batch):
    dev = _device()
    return (batch["token_ids"].long().to(dev), (batch["token_mask"] < 0.5).to(dev),
            batch["token_types"].long().to(dev), batch["seq_len"].long().to(dev),
            batch["reference"])


def _collate(samples):
    out = {k: [s[k] for s in samples] for k in samples[0]}
    for k in ("token_ids", "token_mask", "token_types", "seq_len"):
        out[k] = torch.as_tensor(np.stack(out[k]) if k != "seq_len" else out[k],
                                 dtype=torch.long)
    return out


def get_one_epoch_nq_dataloader(dataset, micro_batch_size=None):
    """Sequential, not distributed, keeps the last partial batch."""
    args = get_args()
    bs = BatchSampler(SequentialSampler(dataset), micro_batch_size or args.micro_batch_size,
                      drop_last=False)
    return DataLoader(dataset, batch_sampler=bs, num_workers=args.num_workers,
                      pin_memory=torch.cuda.is_available(), collate_fn=_collate)


class NQDataset(Dataset):
    def __init__(self, task_name, dataset_name, datapath, tokenizer, max_seq_length):
        self.task_name, self.dataset_name = task_name, dataset_name
        self.tokenizer, self.max_seq_length = tokenizer, max_seq_length
        print_rank_0(f" > building {task_name} dataset for {dataset_name}:")
        self.samples = self.process_samples_from_single_path(datapath)
        print_rank_0(f"  >> total number of samples: {len(self.samples)}")

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, idx):
        s = self.samples[idx]
        ids, types, pad = build_tokens_types_paddings_from_ids(
            self.tokenizer.tokenize(s["question"]), self.max_seq_length, self.tokenizer.cls,
            self.tokenizer.sep, self.tokenizer.pad)
        ids = np.asarray(ids, dtype=np.int64)
        return {"token_ids": ids, "token_mask": make_attention_mask(ids, ids),
                "token_types": np.asarray(types, dtype=np.int64), "seq_len": int(pad.sum()),
                "reference": s["answers"]}

    @staticmethod
    def process_samples_from_single_path(filename):
        print_rank_0(f" > Processing {filename} ...")
        with open(filename, newline="", encoding="utf-8") as f:
            samples = [{"question": r[0], "answers": ast.literal_eval(r[1])}
                       for r in csv.reader(f, delimiter="\t")]
        print_rank_0(f" >> processed {len(samples)} samples.")
        return samples
