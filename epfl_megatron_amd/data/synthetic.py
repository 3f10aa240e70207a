"""Synthetic token datasets (benchmarks / CI without a corpus).

Samples are ``{'text': int64[seq_length + 1]}`` drawn deterministically from a
counter-based generator (sample i is a pure function of (seed, i)), so DP
ranks and resumed runs see reproducible data with no disk I/O — the
throughput benchmark (``bench.py``) measures the model, not the loader.
"""
import numpy as np
import torch


class SyntheticGPTDataset(torch.utils.data.Dataset):
    in_memory = True

    def __init__(self, num_samples, seq_length, vocab_size, seed=1234):
        self.num_samples = int(num_samples)
        self.seq_length = int(seq_length)
        self.vocab_size = int(vocab_size)
        self.seed = int(seed)

    def __len__(self):
        return self.num_samples

    def __getitem__(self, idx):
        rng = np.random.Generator(np.random.Philox(key=self.seed + 0x9E3779B9 * (int(idx) + 1)))
        toks = rng.integers(0, self.vocab_size, size=self.seq_length + 1, dtype=np.int64)
        return {"text": toks}


def synthetic_train_valid_test_datasets(train_valid_test_num_samples, seq_length, vocab_size,
                                        seed=1234):
    out = []
    for i, n in enumerate(train_valid_test_num_samples):
        out.append(SyntheticGPTDataset(max(int(n), 1), seq_length, vocab_size, seed + 7919 * i)
                   if n > 0 else None)
    return tuple(out)
