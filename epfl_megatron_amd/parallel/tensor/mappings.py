"""Tensor/sequence-parallel region boundaries as conjugate autograd pairs.

Semantics follow the reference (``megatron/core/tensor_parallel/mappings.py``):

=========================  ========================  =========================
region op                  forward                   backward
=========================  ========================  =========================
copy_to_tp                 identity                  all-reduce
reduce_from_tp             all-reduce                identity
scatter_to_tp              split last dim            all-gather last dim
gather_from_tp             all-gather last dim       split last dim
scatter_to_sp              split dim 0               all-gather dim 0
gather_from_sp             all-gather dim 0          reduce-scatter (or split)
reduce_scatter_to_sp       reduce-scatter dim 0      all-gather dim 0
=========================  ========================  =========================

The seven pairs are generated from two primitive tables instead of seven
hand-written classes; every collective goes through ``parallel.comm`` so the
same code runs on RCCL (xGMI) and on gloo for CPU tests.
"""
import torch

from .. import state
from .. import comm


def _tp_world():
    return state.get_tensor_model_parallel_world_size()


def _reduce(x):
    if _tp_world() == 1:
        return x
    comm.all_reduce(x, group=state.get_tensor_model_parallel_group())
    return x


def _split_last(x):
    world = _tp_world()
    if world == 1:
        return x
    rank = state.get_tensor_model_parallel_rank()
    return x.chunk(world, dim=-1)[rank].contiguous()


def _split_first(x):
    world = _tp_world()
    if world == 1:
        return x
    if x.shape[0] % world != 0:
        raise AssertionError("first dimension of the tensor should be divisible by tp world size")
    rank = state.get_tensor_model_parallel_rank()
    return x.chunk(world, dim=0)[rank].contiguous()


def _gather_first(x):
    world = _tp_world()
    if world == 1:
        return x
    out = torch.empty((x.shape[0] * world,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    comm.all_gather_into(out, x, group=state.get_tensor_model_parallel_group())
    return out


def _gather_last(x):
    world = _tp_world()
    if world == 1:
        return x
    # Gather along dim 0 of a transposed view, then move the rank axis next to the last dim.
    g = _gather_first(x.movedim(-1, 0).contiguous())
    parts = g.chunk(world, dim=0)
    return torch.cat([p.movedim(0, -1) for p in parts], dim=-1).contiguous()


def _reduce_scatter_first(x):
    world = _tp_world()
    if world == 1:
        return x
    if x.shape[0] % world != 0:
        raise AssertionError("first dimension of the tensor should be divisible by tp world size")
    out = torch.empty((x.shape[0] // world,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    comm.reduce_scatter_into(out, x, group=state.get_tensor_model_parallel_group())
    return out


def _identity(x):
    return x


def _make_pair(name, fwd, bwd):
    class _Fn(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            return fwd(x)

        @staticmethod
        def backward(ctx, g):
            return bwd(g)

    _Fn.__name__ = name
    return _Fn


_CopyToTP = _make_pair("_CopyToTP", _identity, _reduce)
_ReduceFromTP = _make_pair("_ReduceFromTP", _reduce, _identity)
_ScatterToTP = _make_pair("_ScatterToTP", _split_last, _gather_last)
_GatherFromTP = _make_pair("_GatherFromTP", _gather_last, _split_last)
_ScatterToSP = _make_pair("_ScatterToSP", _split_first, _gather_first)
_ReduceScatterToSP = _make_pair("_ReduceScatterToSP", _reduce_scatter_first, _gather_first)


class _GatherFromSP(torch.autograd.Function):
    """All-gather along dim 0; backward reduce-scatters when the consumer's
    grad is TP-partial (the usual case), or just splits otherwise."""

    @staticmethod
    def forward(ctx, x, tensor_parallel_output_grad=True):
        ctx.tp_out_grad = tensor_parallel_output_grad
        return _gather_first(x)

    @staticmethod
    def backward(ctx, g):
        if ctx.tp_out_grad:
            return _reduce_scatter_first(g), None
        return _split_first(g), None


def copy_to_tensor_model_parallel_region(x):
    return _CopyToTP.apply(x)


def reduce_from_tensor_model_parallel_region(x):
    return _ReduceFromTP.apply(x)


def scatter_to_tensor_model_parallel_region(x):
    return _ScatterToTP.apply(x)


def gather_from_tensor_model_parallel_region(x):
    return _GatherFromTP.apply(x)


def scatter_to_sequence_parallel_region(x):
    return _ScatterToSP.apply(x)


def gather_from_sequence_parallel_region(x, tensor_parallel_output_grad=True):
    return _GatherFromSP.apply(x, tensor_parallel_output_grad)


def reduce_scatter_to_sequence_parallel_region(x):
    return _ReduceScatterToSP.apply(x)


# Raw (non-autograd) primitives, exported for layers / p2p / tools.
reduce_tp = _reduce
split_along_last_dim = _split_last
split_along_first_dim = _split_first
gather_along_first_dim = _gather_first
gather_along_last_dim = _gather_last
reduce_scatter_along_first_dim = _reduce_scatter_first
