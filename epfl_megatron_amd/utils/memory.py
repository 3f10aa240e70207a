"""Contiguous bump-allocated buffers (reference ``megatron/memory.py``; unused by
the reference's training path, kept for API parity).

``MemoryBuffer`` hands out views of one flat allocation in order, so a
sequence of same-lifetime tensors lives in a single HBM range; ``reset``
rewinds it.  ``RingMemBuffer`` cycles over N such buffers (e.g. double
buffering of activations across micro-batches).
"""
import operator
from functools import reduce

import torch

_MEM_BUFFS = {}


def allocate_mem_buff(name, numel, dtype, track_usage):
    if name in _MEM_BUFFS:
        raise AssertionError(f"memory buffer {name} already allocated.")
    _MEM_BUFFS[name] = MemoryBuffer(name, numel, dtype, track_usage)
    return _MEM_BUFFS[name]


def get_mem_buff(name):
    return _MEM_BUFFS[name]


class MemoryBuffer:

    def __init__(self, name, numel, dtype, track_usage, device=None):
        if device is None:
            device = torch.cuda.current_device() if torch.cuda.is_available() else "cpu"
        self.name, self.numel, self.dtype = name, numel, dtype
        self.data = torch.empty(numel, dtype=dtype, device=device, requires_grad=False)
        self._start = 0
        self._in_use = False
        self.track_usage = track_usage
        self.in_use_value, self.total_value = 0.0, 0.0

    def reset(self):
        self._start = 0

    def is_in_use(self):
        return self._in_use

    def numel_in_use(self):
        return self._start

    def add(self, tensor):
        """Copy ``tensor`` into the buffer and return the buffer-backed view."""
        if tensor.dtype != self.dtype:
            raise TypeError(f"buffer {self.name} holds {self.dtype}, got {tensor.dtype}")
        view = self.get(tensor.shape)
        view.copy_(tensor)
        return view

    def get(self, shape):
        n = reduce(operator.mul, shape, 1)
        if self._start + n > self.numel:
            raise RuntimeError(f"memory buffer {self.name} out of space "
                               f"({self._start} + {n} > {self.numel})")
        t = self.data[self._start:self._start + n].view(*shape)
        self._start += n
        self._in_use = True
        return t

    def get_data(self):
        self._in_use = False
        if self.track_usage:
            self.in_use_value += float(self._start)
            self.total_value += float(self.numel)
        return self.data[:self._start]

    def print_average_usage(self):
        if not self.track_usage:
            raise AssertionError("usage tracking is off")
        if self.total_value > 0 and torch.distributed.is_initialized() and \
                torch.distributed.get_rank() == 0:
            print(f" > usage of {self.name} memory buffer: "
                  f"{100.0 * self.in_use_value / self.total_value:.2f} %", flush=True)


class RingMemBuffer:

    def __init__(self, name, num_buffers, numel, dtype, track_usage):
        self.num_buffers = num_buffers
        self.buffers = [allocate_mem_buff(f"{name} {i}", numel, dtype, track_usage)
                        for i in range(num_buffers)]
        self._index = -1

    def get_next_buffer(self):
        self._index = (self._index + 1) % self.num_buffers
        buff = self.buffers[self._index]
        if buff.is_in_use():
            raise AssertionError("buffer is already in use.")
        return buff
