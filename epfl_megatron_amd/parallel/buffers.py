"""Reusable activation scratch buffers and view-stripping helpers.

(reference ``megatron/core/utils.py:24-124``).  On MI355X the caching
allocator already recycles blocks cheaply, but gathering the full ``[s, b, h]``
activation for sequence-parallel GEMMs in a named, persistent scratch tensor
avoids allocator fragmentation across the 288 GB pool and keeps the address
stable for hipGraph capture.
"""
import itertools
import operator
from functools import reduce

import torch

_GENERATIONS = itertools.count(1)  # process-wide: never reused across buffer objects


def _use_count(t):
    """References to ``t``'s storage (tensors and views, autograd's saved
    tensors included), measured the same way every time."""
    return torch._C._storage_Use_Count(t.untyped_storage()._cdata)


class GlobalMemoryBuffer:
    """Named scratch tensors, grown on demand and handed out as views.

    Each buffer carries a *generation* that moves whenever the buffer is
    (re)allocated or handed out with a different shape than the previous
    request: two users of one name with different views (e.g. the SP forward's
    ``[c, tp*R, h]`` pieces and the backward's ``[tp*rl, h]`` re-gather) then
    never look like the same contents to code that caches facts about the
    bytes (the simulated-TP loopback all-gather, ``parallel/comm.py``)."""

    def __init__(self):
        self._buffers = {}
        self._last_shape = {}
        self._gen = {}
        self._by_ptr = {}  # storage data_ptr -> key
        self._kept = {}  # get_kept pools: key -> [(buffer, its free use count)]

    def get_tensor(self, shape, dtype, name):
        numel = reduce(operator.mul, shape, 1)
        key = (name, dtype)
        buf = self._buffers.get(key)
        if buf is None or buf.numel() < numel:
            device = torch.cuda.current_device() if torch.cuda.is_available() else "cpu"
            if buf is not None:
                self._by_ptr.pop(buf.untyped_storage().data_ptr(), None)
            buf = torch.empty(numel, dtype=dtype, device=device, requires_grad=False)
            self._buffers[key] = buf
            self._by_ptr[buf.untyped_storage().data_ptr()] = key
            self._last_shape[key] = None
        shape = tuple(shape)
        if self._last_shape.get(key) != shape:
            self._last_shape[key] = shape
            self._gen[key] = next(_GENERATIONS)
        return buf[:numel].view(*shape)

    def get_kept(self, shape, dtype, device):
        """A tensor for an SP gather that is kept for the backward under the
        simulated-TP loopback (``parallel/comm.py``): taken from a pool of
        persistent buffers, one not referenced by anything but the pool (its
        storage use count back at the pool's own), else a new one.  Registered
        like the named buffers, with a generation fixed per buffer, so the
        loopback all-gather fills the simulated peers' slots once per buffer
        instead of on every call (the fresh allocation a real run uses would be
        rewritten whole each time: 7/8 of the gathered bytes of extra copies
        per call at TP = 8, ~3 % of the 7B TP8 proxy step)."""
        shape = tuple(shape)
        key = ("kept", shape, dtype, str(device))
        pool = self._kept.setdefault(key, [])
        for buf, base in pool:
            if _use_count(buf) == base:
                return buf.view(*shape)
        buf = torch.empty(shape, dtype=dtype, device=device)
        bkey = key + (len(pool),)
        self._by_ptr[buf.untyped_storage().data_ptr()] = bkey
        self._gen[bkey] = next(_GENERATIONS)
        pool.append((buf, _use_count(buf)))
        return buf.view(*shape)

    def owner(self, t):
        """``(key, generation)`` of the scratch buffer holding ``t``, or None
        (one dict lookup by storage address)."""
        key = self._by_ptr.get(t.untyped_storage().data_ptr())
        return None if key is None else (key, self._gen[key])


_GLOBAL_BUFFER = None


def get_global_memory_buffer():
    global _GLOBAL_BUFFER
    if _GLOBAL_BUFFER is None:
        _GLOBAL_BUFFER = GlobalMemoryBuffer()
    return _GLOBAL_BUFFER


def reset_global_memory_buffer():
    global _GLOBAL_BUFFER
    _GLOBAL_BUFFER = None


def _kernel_make_viewless_tensor(inp, requires_grad):
    out = torch.empty((1,), dtype=inp.dtype, device=inp.device, requires_grad=requires_grad)
    out.data = inp.data
    return out


class MakeViewlessTensor(torch.autograd.Function):
    @staticmethod
    def forward(ctx, inp, requires_grad):
        return _kernel_make_viewless_tensor(inp, requires_grad)

    @staticmethod
    def backward(ctx, grad_output):
        return grad_output, None


def make_viewless_tensor(inp, requires_grad, keep_graph):
    """Return a tensor sharing ``inp``'s storage whose ``._base`` is None, so
    that pipeline "pseudo-free" of outputs actually releases memory."""
    if inp._base is None:
        return inp
    if keep_graph:
        return MakeViewlessTensor.apply(inp, requires_grad)
    return _kernel_make_viewless_tensor(inp, requires_grad)


def assert_viewless_tensor(tensor, extra_msg=None):
    if isinstance(tensor, (list, tuple)):
        for t in tensor:
            assert_viewless_tensor(t, extra_msg)
        return tensor
    if not isinstance(tensor, torch.Tensor):
        return tensor
    if tensor._base is not None:
        raise AssertionError("Ensure tensor._base is None before setting tensor.data or "
                             f"storing tensor to memory buffer. Found tensor._base={tensor._base}. "
                             f"{extra_msg or ''}")
    return tensor


def safely_set_viewless_tensor_data(tensor, new_data_tensor):
    assert_viewless_tensor(tensor, extra_msg="FYI, tensor._base has shape "
                           f"{'--' if tensor._base is None else tensor._base.shape}")
    tensor.data = new_data_tensor


def divide(numerator, denominator):
    if numerator % denominator != 0:
        raise AssertionError(f"{numerator} is not divisible by {denominator}")
    return numerator // denominator
