"""RACE reading comprehension (reference ``tasks/race/data.py``).

Every ``*.txt`` under a split directory holds one JSON document per line
(``article``, ``questions``, ``options``, ``answers``).  Each question becomes
one sample of ``NUM_CHOICES`` rows ``[CLS] question+choice [SEP] article
[SEP]``; a ``_`` in the question is a cloze slot filled by the choice.  The
dataset advertises ``sample_multiplier = 4`` so the finetune driver scales
micro/global batch sizes to the expanded batch dimension.
"""
import glob
import json
import os
import time

from torch.utils.data import Dataset

from epfl_megatron_amd import print_rank_0

from ..data_utils import build_sample, build_tokens_types_paddings_from_ids, clean_text

NUM_CHOICES = 4
MAX_QA_LENGTH = 128


class RaceDataset(Dataset):
    def __init__(self, dataset_name, datapaths, tokenizer, max_seq_length,
                 max_qa_length=MAX_QA_LENGTH):
        self.dataset_name = dataset_name
        print_rank_0(f" > building RACE dataset for {dataset_name}:")
        print_rank_0("  > paths: " + " ".join(datapaths))
        self.samples = []
        for p in datapaths:
            self.samples.extend(process_single_datapath(p, tokenizer, max_qa_length,
                                                        max_seq_length))
        print_rank_0(f"  >> total number of samples: {len(self.samples)}")
        self.sample_multiplier = NUM_CHOICES

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, idx):
        return self.samples[idx]


def process_single_datapath(datapath, tokenizer, max_qa_length, max_seq_length):
    t0 = time.time()
    samples, n_docs, n_q = [], 0, 0
    for fn in sorted(glob.glob(os.path.join(datapath, "*.txt"))):
        with open(fn, "r", encoding="utf-8") as f:
            for line in f:
                d = json.loads(line)
                n_docs += 1
                qs, opts, answers = d["questions"], d["options"], d["answers"]
                assert len(qs) == len(answers) == len(opts)
                ctx_ids = tokenizer.tokenize(clean_text(d["article"]))
                for q, choices, ans in zip(qs, opts, answers):
                    n_q += 1
                    label = ord(ans) - ord("A")
                    assert 0 <= label < NUM_CHOICES and len(choices) == NUM_CHOICES
                    rows = []
                    for c in choices:
                        qa = q.replace("_", c) if "_" in q else " ".join([q, c])
                        qa_ids = tokenizer.tokenize(clean_text(qa))[:max_qa_length]
                        rows.append(build_tokens_types_paddings_from_ids(
                            qa_ids, ctx_ids, max_seq_length, tokenizer.cls, tokenizer.sep,
                            tokenizer.pad))
                    ids, types, pads = zip(*rows)
                    samples.append(build_sample(ids, types, pads, label, len(samples)))
    print_rank_0(f"    > processed {n_docs} document, {n_q} questions, and {len(samples)} "
                 f"samples in {time.time() - t0:.2f} seconds")
    return samples
