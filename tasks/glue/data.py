"""GLUE sentence-pair datasets (reference ``tasks/glue/{data,mnli,qqp}.py``).

Each reader turns one TSV file into ``{"text_a", "text_b", "label", "uid"}``
records; ``__getitem__`` tokenizes lazily into the ``[CLS] a [SEP] b [SEP]``
layout.  A header row of the test-split shape (MNLI: 10 columns, QQP: 3)
switches the reader to test mode, where every record gets ``test_label``.
"""
from torch.utils.data import Dataset

from epfl_megatron_amd import print_rank_0

from ..data_utils import build_sample, build_tokens_types_paddings_from_text, clean_text


class GLUEAbstractDataset(Dataset):
    task_name = "GLUE"

    def __init__(self, dataset_name, datapaths, tokenizer, max_seq_length):
        self.dataset_name = dataset_name
        self.tokenizer = tokenizer
        self.max_seq_length = max_seq_length
        print_rank_0(f" > building {self.task_name} dataset for {dataset_name}:")
        print_rank_0("  > paths: " + " ".join(datapaths))
        self.samples = []
        for p in datapaths:
            self.samples.extend(self.process_samples_from_single_path(p))
        print_rank_0(f"  >> total number of samples: {len(self.samples)}")

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, idx):
        s = self.samples[idx]
        ids, types, pads = build_tokens_types_paddings_from_text(
            s["text_a"], s["text_b"], self.tokenizer, self.max_seq_length)
        return build_sample(ids, types, pads, s["label"], s["uid"])

    def process_samples_from_single_path(self, path):
        raise NotImplementedError

    @staticmethod
    def _rows(path):
        with open(path, "r", encoding="utf-8") as f:
            for line in f:
                yield line.strip().split("\t")


class MNLIDataset(GLUEAbstractDataset):
    """MultiNLI: columns 8/9 are the sentence pair, the last is the gold label."""
    task_name = "MNLI"
    LABELS = {"contradiction": 0, "entailment": 1, "neutral": 2}

    def __init__(self, name, datapaths, tokenizer, max_seq_length, test_label="contradiction"):
        self.test_label = test_label
        super().__init__(name, datapaths, tokenizer, max_seq_length)

    def process_samples_from_single_path(self, path):
        print_rank_0(f" > Processing {path} ...")
        rows = self._rows(path)
        header = next(rows)
        is_test = len(header) == 10
        out = []
        for row in rows:
            label = self.test_label if is_test else row[-1].strip()
            s = {"text_a": clean_text(row[8].strip()), "text_b": clean_text(row[9].strip()),
                 "uid": int(row[0].strip())}
            assert s["text_a"] and s["text_b"] and label in self.LABELS and s["uid"] >= 0
            s["label"] = self.LABELS[label]
            out.append(s)
        print_rank_0(f" >> processed {len(out)} samples.")
        return out


class QQPDataset(GLUEAbstractDataset):
    """Quora Question Pairs: ``id qid1 qid2 q1 q2 is_duplicate`` (test: ``id q1 q2``).
    Malformed or empty training rows are skipped with a warning."""
    task_name = "QQP"
    LABELS = (0, 1)

    def __init__(self, name, datapaths, tokenizer, max_seq_length, test_label=0):
        self.test_label = test_label
        super().__init__(name, datapaths, tokenizer, max_seq_length)

    def process_samples_from_single_path(self, path):
        print_rank_0(f" > Processing {path} ...")
        rows = self._rows(path)
        header = next(rows)
        is_test = len(header) == 3
        assert is_test or len(header) == 6
        out = []
        for row in rows:
            if is_test:
                assert len(row) == 3, f"expected length 3: {row}"
                uid, a, b, label = int(row[0]), clean_text(row[1].strip()), \
                    clean_text(row[2].strip()), self.test_label
                assert a and b
            else:
                if len(row) != 6:
                    print_rank_0(f"***WARNING*** index error, skipping: {row}")
                    continue
                uid, a, b = int(row[0]), clean_text(row[3].strip()), clean_text(row[4].strip())
                label = int(row[5].strip())
                if not a or not b:
                    print_rank_0(f"***WARNING*** zero length text, skipping: {row}")
                    continue
            assert label in self.LABELS and uid >= 0
            out.append({"uid": uid, "text_a": a, "text_b": b, "label": label})
        print_rank_0(f" >> processed {len(out)} samples.")
        return out
