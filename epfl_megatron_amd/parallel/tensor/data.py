"""TP-rank-0 broadcast of a batch dict (reference ``core/tensor_parallel/data.py``).

Only TP-rank 0 reads the dataset; it broadcasts sizes (one int64 vector)
then one flat payload per dtype to the rest of its TP group.

Host->device: the flat payload is staged in a small ring of pinned host
buffers and copied with ``non_blocking=True``, so feeding a micro-batch never
blocks the host on the GPU queue.  Without TP there is nothing to broadcast and
the sizes come straight from the host tensors (no size round trip).

Under TP the receiving ranks need the shapes on the HOST to size the payload,
and reading a broadcast size vector back drains the GPU queue.  So the sizes
are broadcast once per key set and then reused (every micro-batch of a run has
the same shapes); only ``--variable_seq_lengths`` re-broadcasts them each call.
TP-rank 0 checks its real shapes against the cached ones and raises rather
than let the group post mismatched broadcasts.  Both broadcasts go through
``parallel/comm.py`` (accounted as ``broadcast/tp``).
"""
import torch

from .. import comm, state

_MAX_DATA_DIM = 5


def _device():
    return torch.cuda.current_device() if torch.cuda.is_available() else "cpu"


class _PinnedRing:
    """Reusable pinned staging buffers; a slot is reused only after the copy
    that last read it has completed (event), which in steady state is long
    before the ring wraps."""

    def __init__(self, slots=4):
        self.slots = [None] * slots
        self.events = [None] * slots
        self.i = 0

    def to_device(self, cpu_flat, device):
        if not torch.cuda.is_available() or device == "cpu":
            return cpu_flat
        k = self.i
        self.i = (self.i + 1) % len(self.slots)
        buf = self.slots[k]
        n = cpu_flat.numel()
        if buf is None or buf.numel() < n or buf.dtype != cpu_flat.dtype:
            buf = torch.empty(max(n, 1), dtype=cpu_flat.dtype, pin_memory=True)
            self.slots[k], self.events[k] = buf, None
        if self.events[k] is not None:
            self.events[k].synchronize()
        buf[:n].copy_(cpu_flat)
        out = buf[:n].to(device, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.events[k] = ev
        return out


_RING = _PinnedRing()


def _build_key_size_numel_dictionaries(keys, data):
    sizes = [0] * (_MAX_DATA_DIM * len(keys))
    if state.get_tensor_model_parallel_rank() == 0:
        for i, key in enumerate(keys):
            shape = data[key].size()
            if len(shape) >= _MAX_DATA_DIM:
                raise AssertionError("you should increase MAX_DATA_DIM")
            for j, d in enumerate(shape):
                sizes[i * _MAX_DATA_DIM + j] = d
    sizes_t = torch.tensor(sizes, dtype=torch.long, device=_device())
    if state.get_tensor_model_parallel_world_size() > 1:
        comm.broadcast(sizes_t, state.get_tensor_model_parallel_src_rank(),
                       group=state.get_tensor_model_parallel_group())
    sizes_cpu = sizes_t.cpu().tolist()  # the one host sync (first call per key set)
    key_size, key_numel, total = {}, {}, 0
    for i, key in enumerate(keys):
        shape = []
        for j in range(_MAX_DATA_DIM):
            d = sizes_cpu[i * _MAX_DATA_DIM + j]
            if d == 0:
                break
            shape.append(d)
        numel = 1
        for d in shape:
            numel *= d
        key_size[key], key_numel[key] = shape, numel
        total += numel
    return key_size, key_numel, total


def _local_sizes(keys, data):
    key_size, key_numel, total = {}, {}, 0
    for key in keys:
        shape = list(data[key].size())
        if len(shape) >= _MAX_DATA_DIM:
            raise AssertionError("you should increase MAX_DATA_DIM")
        n = 1
        for d in shape:
            n *= d
        key_size[key], key_numel[key] = shape, n
        total += n
    return key_size, key_numel, total


_SIZE_CACHE = {}  # (tuple(keys), id(tp group)) -> (key_size, key_numel, total)


def _variable_lengths():
    from ...global_vars import get_args_or_none
    args = get_args_or_none()
    return bool(getattr(args, "variable_seq_lengths", False))


def reset_size_cache():
    _SIZE_CACHE.clear()


def broadcast_data(keys, data, datatype):
    if state.get_tensor_model_parallel_world_size() == 1:
        key_size, key_numel, total = _local_sizes(keys, data)
    else:
        ck = (tuple(keys), id(state.get_tensor_model_parallel_group()))
        hit = None if _variable_lengths() else _SIZE_CACHE.get(ck)
        if hit is None:
            hit = _SIZE_CACHE[ck] = _build_key_size_numel_dictionaries(keys, data)
        elif state.get_tensor_model_parallel_rank() == 0:
            for key in keys:
                if list(data[key].size()) != hit[0][key]:
                    raise RuntimeError(
                        f"broadcast_data: '{key}' has shape {list(data[key].size())} but this "
                        f"run's batches had {hit[0][key]}; shapes are broadcast once per run "
                        "unless --variable_seq_lengths is set")
        key_size, key_numel, total = hit
    if state.get_tensor_model_parallel_rank() == 0:
        for key in keys:
            if data[key].dtype != datatype:
                raise AssertionError(f"{key} has data type {data[key].dtype} which is different "
                                     f"than {datatype}")
        flat = torch.cat([data[k].contiguous().view(-1) for k in keys], dim=0)
        flat = _RING.to_device(flat, _device()) if not flat.is_cuda else flat
    else:
        flat = torch.empty(total, device=_device(), dtype=datatype)
    if state.get_tensor_model_parallel_world_size() > 1:
        comm.broadcast(flat, state.get_tensor_model_parallel_src_rank(),
                       group=state.get_tensor_model_parallel_group())
    out, offset = {}, 0
    for key in keys:
        n = key_numel[key]
        out[key] = flat.narrow(0, offset, n).view(key_size[key])
        offset += n
    return out
