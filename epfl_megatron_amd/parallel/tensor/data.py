"""TP-rank-0 broadcast of a batch dict (reference ``core/tensor_parallel/data.py``).

Only TP-rank 0 reads the dataset; it broadcasts sizes (one int64 vector)
then one flat payload per dtype to the rest of its TP group.
"""
import torch
import torch.distributed as dist

from .. import state

_MAX_DATA_DIM = 5


def _device():
    return torch.cuda.current_device() if torch.cuda.is_available() else "cpu"


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
        dist.broadcast(sizes_t, state.get_tensor_model_parallel_src_rank(),
                       group=state.get_tensor_model_parallel_group())
    sizes_cpu = sizes_t.cpu().tolist()
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


def broadcast_data(keys, data, datatype):
    key_size, key_numel, total = _build_key_size_numel_dictionaries(keys, data)
    if state.get_tensor_model_parallel_rank() == 0:
        for key in keys:
            if data[key].dtype != datatype:
                raise AssertionError(f"{key} has data type {data[key].dtype} which is different "
                                     f"than {datatype}")
        flat = torch.cat([data[k].contiguous().view(-1) for k in keys], dim=0).to(_device())
    else:
        flat = torch.empty(total, device=_device(), dtype=datatype)
    if state.get_tensor_model_parallel_world_size() > 1:
        dist.broadcast(flat, state.get_tensor_model_parallel_src_rank(),
                       group=state.get_tensor_model_parallel_group())
    out, offset = {}, 0
    for key in keys:
        n = key_numel[key]
        out[key] = flat.narrow(0, offset, n).view(key_size[key])
        offset += n
    return out
