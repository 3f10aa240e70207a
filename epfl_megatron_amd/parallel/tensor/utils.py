"""Small tensor-parallel helpers (reference ``core/tensor_parallel/utils.py``)."""
import torch

from .. import state, comm
from ..buffers import divide


def split_tensor_along_last_dim(tensor, num_partitions, contiguous_split_chunks=False):
    last = divide(tensor.size(-1), num_partitions)
    chunks = torch.split(tensor, last, dim=-1)
    if contiguous_split_chunks:
        return tuple(c.contiguous() for c in chunks)
    return chunks


def split_tensor_into_1d_equal_chunks(tensor, new_buffer=False):
    """This TP rank's 1/tp slice of the flattened tensor."""
    world = state.get_tensor_model_parallel_world_size()
    per = divide(tensor.numel(), world)
    start = per * state.get_tensor_model_parallel_rank()
    flat = tensor.view(-1)[start:start + per]
    if new_buffer:
        out = torch.empty(per, dtype=tensor.dtype, device=tensor.device, requires_grad=False)
        out.copy_(flat)
        return out
    return flat


def gather_split_1d_tensor(tensor):
    """Inverse of :func:`split_tensor_into_1d_equal_chunks` (all-gather over TP)."""
    world = state.get_tensor_model_parallel_world_size()
    out = torch.empty(tensor.numel() * world, dtype=tensor.dtype, device=tensor.device,
                      requires_grad=False)
    comm.all_gather_into(out, tensor, group=state.get_tensor_model_parallel_group())
    return out


class VocabUtility:
    """Vocab range ``[first, last)`` owned by a TP rank."""

    @staticmethod
    def vocab_range_from_per_partition_vocab_size(per_partition_vocab_size, rank, world_size):
        first = rank * per_partition_vocab_size
        return first, first + per_partition_vocab_size

    @staticmethod
    def vocab_range_from_global_vocab_size(global_vocab_size, rank, world_size):
        per = divide(global_vocab_size, world_size)
        return VocabUtility.vocab_range_from_per_partition_vocab_size(per, rank, world_size)
