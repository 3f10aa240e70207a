"""Weighted mixture of datasets (reference ``megatron/data/blendable_dataset.py:12``).

Sample ``i`` comes from dataset ``dataset_index[i]``, position
``dataset_sample_index[i]``; the interleave is the native greedy
largest-deficit schedule (``helpers.build_blending_indices``), so the achieved
proportions track the weights at every prefix of the stream.
"""
import time

import numpy as np
import torch

from ..utils.misc import print_rank_0
from . import helpers


def _is_rank0():
    return not torch.distributed.is_initialized() or torch.distributed.get_rank() == 0


class BlendableDataset(torch.utils.data.Dataset):

    def __init__(self, datasets, weights):
        if len(datasets) != len(weights):
            raise ValueError("one weight per dataset")
        if len(datasets) >= 255:
            raise ValueError("at most 254 datasets can be blended")
        self.datasets = datasets
        self.size = sum(len(d) for d in datasets)
        w = np.asarray(weights, dtype=np.float64)
        if w.sum() <= 0:
            raise ValueError("blend weights must sum to a positive value")
        w = w / w.sum()
        t0 = time.time()
        self.dataset_index = np.zeros(self.size, dtype=np.uint8)
        self.dataset_sample_index = np.zeros(self.size, dtype=np.int64)
        helpers.build_blending_indices(self.dataset_index, self.dataset_sample_index, w,
                                       len(datasets), self.size, _is_rank0())
        print_rank_0(f"> elapsed time for building blendable dataset indices: "
                     f"{time.time() - t0:.2f} (sec)")

    def __len__(self):
        return self.size

    def __getitem__(self, idx):
        return self.datasets[self.dataset_index[idx]][int(self.dataset_sample_index[idx])]
