"""Resumable batch samplers (reference ``megatron/data/data_samplers.py``).

Each step consumes ``global_batch`` consecutive sample ids starting at
``consumed_samples``; within each ``micro_batch * dp`` window DP rank r takes
``[r * mbs, (r + 1) * mbs)``.
"""
import random

import numpy as np
import torch

from .. import global_vars
from ..parallel import state


def build_pretraining_data_loader(dataset, consumed_samples):
    if dataset is None:
        return None
    args = global_vars.get_args()
    # context-parallel ranks of one DP group read the same samples
    dp_rank = state.get_data_sample_parallel_rank()
    dp_size = state.get_data_sample_parallel_world_size()
    if args.dataloader_type == "single":
        sampler = MegatronPretrainingSampler(len(dataset), consumed_samples, args.micro_batch_size,
                                             dp_rank, dp_size)
    elif args.dataloader_type == "cyclic":
        sampler = MegatronPretrainingRandomSampler(dataset, len(dataset), consumed_samples,
                                                   args.micro_batch_size, dp_rank, dp_size,
                                                   args.data_sharding)
    else:
        raise Exception(f"{args.dataloader_type} dataloader type is not supported.")
    workers = args.num_workers if not getattr(dataset, "in_memory", False) else 0
    return torch.utils.data.DataLoader(dataset, batch_sampler=sampler, num_workers=workers,
                                       pin_memory=torch.cuda.is_available(),
                                       persistent_workers=workers > 0)


class MegatronPretrainingSampler:
    def __init__(self, total_samples, consumed_samples, micro_batch_size, data_parallel_rank,
                 data_parallel_size, drop_last=True):
        if total_samples <= 0:
            raise AssertionError(f"no sample to consume: {total_samples}")
        if consumed_samples >= total_samples:
            raise AssertionError(f"no samples left to consume: {consumed_samples}, {total_samples}")
        if micro_batch_size <= 0 or data_parallel_size <= 0:
            raise AssertionError("invalid batch / dp sizes")
        if data_parallel_rank >= data_parallel_size:
            raise AssertionError("data_parallel_rank should be smaller than data size")
        self.total_samples = total_samples
        self.consumed_samples = consumed_samples
        self.micro_batch_size = micro_batch_size
        self.data_parallel_rank = data_parallel_rank
        self.window = micro_batch_size * data_parallel_size
        self.drop_last = drop_last

    def __len__(self):
        return self.total_samples

    def _my_slice(self):
        s = self.data_parallel_rank * self.micro_batch_size
        return s, s + self.micro_batch_size

    def __iter__(self):
        batch = []
        for idx in range(self.consumed_samples, self.total_samples):
            batch.append(idx)
            if len(batch) == self.window:
                s, e = self._my_slice()
                yield batch[s:e]
                batch = []
        if batch and not self.drop_last:
            s, e = self._my_slice()
            yield batch[s:e]


class RandomSeedDataset(torch.utils.data.Dataset):
    """Reseed python/numpy/torch per sample (seed + idx) for image-style datasets."""

    def __init__(self, dataset):
        args = global_vars.get_args()
        self.base_seed = args.seed
        self.curr_seed = args.seed
        self.dataset = dataset

    def __len__(self):
        return len(self.dataset)

    def set_epoch(self, epoch):
        self.curr_seed = self.base_seed + epoch

    def __getitem__(self, idx):
        seed = idx + self.curr_seed
        torch.manual_seed(seed)
        random.seed(seed)
        np.random.seed(seed)
        return self.dataset[idx]


class MegatronPretrainingRandomSampler:
    """Per-epoch random permutation (seeded by epoch), resumable mid-epoch."""

    def __init__(self, dataset, total_samples, consumed_samples, micro_batch_size,
                 data_parallel_rank, data_parallel_size, data_sharding=True):
        self.dataset = dataset
        self.total_samples = total_samples
        self.consumed_samples = consumed_samples
        self.micro_batch_size = micro_batch_size
        self.data_parallel_rank = data_parallel_rank
        self.data_parallel_size = data_parallel_size
        self.data_sharding = data_sharding
        self.window = micro_batch_size * data_parallel_size
        self.last_batch_size = self.total_samples % self.window
        if total_samples <= 0 or micro_batch_size <= 0 or data_parallel_rank >= data_parallel_size:
            raise AssertionError("invalid sampler configuration")

    def __len__(self):
        return self.total_samples

    def __iter__(self):
        active = self.total_samples - self.last_batch_size
        epoch = self.consumed_samples // active
        current = self.consumed_samples % active
        if isinstance(self.dataset, RandomSeedDataset):
            self.dataset.set_epoch(epoch)
        g = torch.Generator()
        g.manual_seed(epoch)
        if self.data_sharding:
            bucket = (self.total_samples // self.window) * self.micro_batch_size
            offset = current // self.data_parallel_size
            start = self.data_parallel_rank * bucket
            perm = torch.randperm(bucket, generator=g).tolist()
            idx_range = [start + x for x in perm[offset:]]
        else:
            full = (self.total_samples // self.micro_batch_size) * self.micro_batch_size
            perm = torch.randperm(full, generator=g).tolist()
            idx_range = perm[current:][self.data_parallel_rank::self.data_parallel_size]
        batch = []
        for idx in idx_range:
            batch.append(idx)
            if len(batch) == self.micro_batch_size:
                self.consumed_samples += self.window
                yield batch
                batch = []
