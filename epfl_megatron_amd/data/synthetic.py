"""Synthetic token datasets (benchmarks / CI without a corpus).

Samples are ``{'text': int64[seq_length + 1]}`` drawn deterministically from a
counter-based generator (sample i is a pure function of (seed, i)), so DP
ranks and resumed runs see reproducible data with no disk I/O — the
throughput benchmark (``bench.py``) measures the model, not the loader.

``pattern``:
  * ``uniform`` — i.i.d. uniform tokens (loss stays at ln V: nothing to learn);
  * ``cycle``   — a walk along one fixed random cyclic permutation of the
    vocabulary (next token = a fixed function of the current one) from a random
    start.  Same shapes and cost, but learnable: a falling loss in a few steps
    is end-to-end evidence that forward, backward and the optimizer are right.
"""
import numpy as np
import torch


class SyntheticGPTDataset(torch.utils.data.Dataset):
    in_memory = True

    def __init__(self, num_samples, seq_length, vocab_size, seed=1234, pattern="uniform"):
        self.num_samples = int(num_samples)
        self.seq_length = int(seq_length)
        self.vocab_size = int(vocab_size)
        self.seed = int(seed)
        if pattern not in ("uniform", "cycle"):
            raise ValueError(f"unknown synthetic pattern {pattern!r}")
        self.pattern = pattern
        if pattern == "cycle":
            # shared by train/valid/test (same "language"), independent of ``seed``
            order = np.random.default_rng(20240601).permutation(self.vocab_size)
            reps = (self.seq_length + 1) // self.vocab_size + 2
            self._walk = np.tile(order, reps).astype(np.int64)

    def __len__(self):
        return self.num_samples

    def __getitem__(self, idx):
        rng = np.random.Generator(np.random.Philox(key=self.seed + 0x9E3779B9 * (int(idx) + 1)))
        if self.pattern == "cycle":
            j = int(rng.integers(0, self.vocab_size))
            return {"text": self._walk[j:j + self.seq_length + 1].copy()}
        toks = rng.integers(0, self.vocab_size, size=self.seq_length + 1, dtype=np.int64)
        return {"text": toks}


def synthetic_train_valid_test_datasets(train_valid_test_num_samples, seq_length, vocab_size,
                                        seed=1234, pattern="uniform"):
    out = []
    for i, n in enumerate(train_valid_test_num_samples):
        out.append(SyntheticGPTDataset(max(int(n), 1), seq_length, vocab_size, seed + 7919 * i,
                                       pattern=pattern)
                   if n > 0 else None)
    return tuple(out)
