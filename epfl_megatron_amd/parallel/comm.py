"""Collective helpers.

On MI355X every collective here runs on RCCL (the ``nccl`` backend name in
PyTorch-ROCm) over xGMI.  The CPU plumbing path (BASELINE config #1) runs the
same code on ``gloo``, which lacks the fused tensor collectives; the helpers
below pick the tensor form when the backend has it and an equivalent
list-based form otherwise.  Nothing here changes *what* is communicated.
"""
import torch
import torch.distributed as dist


def _is_gloo(group):
    try:
        return dist.get_backend(group) == "gloo"
    except Exception:  # pragma: no cover - uninitialized
        return False


def all_gather_into(output, inp, group, async_op=False):
    """``output`` = concat over ranks of ``inp`` along dim 0."""
    if _is_gloo(group):
        world = dist.get_world_size(group)
        chunks = list(output.chunk(world, dim=0))
        tmp = [torch.empty_like(c) for c in chunks]
        dist.all_gather(tmp, inp.contiguous(), group=group)
        for c, t in zip(chunks, tmp):
            c.copy_(t)
        return None
    return dist.all_gather_into_tensor(output, inp.contiguous(), group=group, async_op=async_op)


def reduce_scatter_into(output, inp, group, async_op=False, op=dist.ReduceOp.SUM):
    """``output`` = this rank's dim-0 chunk of the sum over ranks of ``inp``."""
    if _is_gloo(group):
        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        tmp = inp.contiguous().clone()
        dist.all_reduce(tmp, op=op, group=group)
        output.copy_(tmp.chunk(world, dim=0)[rank])
        return None
    return dist.reduce_scatter_tensor(output, inp.contiguous(), op=op, group=group,
                                      async_op=async_op)


def all_reduce(tensor, group, async_op=False, op=dist.ReduceOp.SUM):
    return dist.all_reduce(tensor, op=op, group=group, async_op=async_op)
