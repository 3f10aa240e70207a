"""Process-group topology for TP x DP x PP.

Rank layout contract (reference ``megatron/core/parallel_state.py:51-199``):
``global_rank = pp_rank * (tp * dp) + dp_rank * tp + tp_rank`` — tensor
parallel ranks are contiguous (so a TP group stays on one node's xGMI mesh),
data parallel is the middle axis and pipeline stages are strided by
``world / pp``.  We build the whole grid once as a ``[pp, dp, tp]`` array and
slice groups out of it, instead of nested rank loops.

Public getters keep the reference names so model/optimizer code reads the
same; a ``set_*`` override layer lets offline tools fake a topology without
``torch.distributed`` (used by the checkpoint re-sharder).
"""

from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np
import torch
import torch.distributed as dist


@dataclass
class _State:
    tp_group: Optional[object] = None
    pp_group: Optional[object] = None
    dp_group: Optional[object] = None
    mp_group: Optional[object] = None
    embedding_group: Optional[object] = None
    position_embedding_group: Optional[object] = None
    embedding_ranks: List[int] = field(default_factory=list)
    position_embedding_ranks: List[int] = field(default_factory=list)
    pp_global_ranks: List[int] = field(default_factory=list)
    dp_global_ranks: List[int] = field(default_factory=list)
    # extra communicators over the same DP ranks (one RCCL stream each)
    dp_comm_groups: List[object] = field(default_factory=list)
    tp_global_ranks: List[int] = field(default_factory=list)
    # context parallelism: consecutive DP indices share one sequence
    cp_group: Optional[object] = None
    cp_size: int = 1
    virtual_pp_rank: Optional[int] = None
    virtual_pp_world_size: Optional[int] = None
    pp_split_rank: Optional[int] = None
    # Overrides (tools that build per-rank models in one process).
    tp_world_override: Optional[int] = None
    pp_world_override: Optional[int] = None
    tp_rank_override: Optional[int] = None
    pp_rank_override: Optional[int] = None
    grid: Optional[np.ndarray] = None


_S = _State()


def rank_grid(world_size, tp, pp):
    """``grid[p, d, t]`` = global rank with pipeline stage p, DP index d, TP index t."""
    if world_size % (tp * pp) != 0:
        raise RuntimeError(f"world_size ({world_size}) is not divisible by tp ({tp}) x pp ({pp})")
    dp = world_size // (tp * pp)
    return np.arange(world_size).reshape(pp, dp, tp)


def _new_group(ranks, backend=None):
    ranks = [int(r) for r in ranks]
    return dist.new_group(ranks, backend=backend) if backend else dist.new_group(ranks)


def initialize_model_parallel(tensor_model_parallel_size=1,
                              pipeline_model_parallel_size=1,
                              virtual_pipeline_model_parallel_size=None,
                              pipeline_model_parallel_split_rank=None,
                              data_parallel_comm_groups=1,
                              context_parallel_size=1):
    """Create TP/DP/PP/model-parallel/embedding groups.

    Every rank must call ``new_group`` for every group in the same order
    (a torch.distributed requirement), so we iterate the full grid on all ranks.
    ``data_parallel_comm_groups`` > 1 adds communicators over the same DP ranks:
    each has its own RCCL stream, so the DDP buckets assigned round-robin to
    them are reduced concurrently.
    ``context_parallel_size`` C > 1 subdivides every DP group: C consecutive
    DP indices (each TP / PP coordinate fixed) hold the C sequence chunks of
    the same samples and form one context-parallel group (``parallel/context.py``
    ring attention).  Gradients are still reduced over the whole DP group;
    the data loader shards samples over DP / C.
    """
    if not dist.is_initialized():
        raise RuntimeError("torch.distributed must be initialized first")
    world = dist.get_world_size()
    rank = dist.get_rank()
    tp, pp = tensor_model_parallel_size, pipeline_model_parallel_size
    grid = rank_grid(world, tp, pp)
    npp, ndp, ntp = grid.shape
    if virtual_pipeline_model_parallel_size is not None:
        _S.virtual_pp_rank = 0
        _S.virtual_pp_world_size = virtual_pipeline_model_parallel_size
    if pipeline_model_parallel_split_rank is not None:
        _S.pp_split_rank = pipeline_model_parallel_split_rank
    _S.grid = grid

    # Data-parallel groups: fix (pp, tp), vary dp.
    if _S.dp_group is not None:
        raise RuntimeError("data parallel group is already initialized")
    for p in range(npp):
        for t in range(ntp):
            ranks = grid[p, :, t]
            g = _new_group(ranks)
            if rank in ranks:
                _S.dp_group, _S.dp_global_ranks = g, [int(r) for r in ranks]
    _S.dp_comm_groups = [_S.dp_group]
    cp = int(context_parallel_size or 1)
    if ndp % cp != 0:
        raise RuntimeError(f"data parallel size ({ndp}) is not divisible by context parallel "
                           f"size ({cp})")
    _S.cp_size = cp
    for p in range(npp):
        for t in range(ntp):
            for c0 in range(0, ndp, cp):
                ranks = grid[p, c0:c0 + cp, t]
                g = _new_group(ranks) if cp > 1 else None
                if rank in ranks:
                    _S.cp_group = g
    for _ in range(max(1, int(data_parallel_comm_groups)) - 1):
        for p in range(npp):
            for t in range(ntp):
                ranks = grid[p, :, t]
                g = _new_group(ranks)
                if rank in ranks:
                    _S.dp_comm_groups.append(g)
    # Model-parallel groups: fix dp, vary (pp, tp).
    for d in range(ndp):
        ranks = grid[:, d, :].reshape(-1)
        g = _new_group(ranks)
        if rank in ranks:
            _S.mp_group = g
    # Tensor-parallel groups: contiguous ranks.
    for p in range(npp):
        for d in range(ndp):
            ranks = grid[p, d, :]
            g = _new_group(ranks)
            if rank in ranks:
                _S.tp_group, _S.tp_global_ranks = g, [int(r) for r in ranks]
    # Pipeline groups (strided) + embedding groups {first, [split], last}.
    for d in range(ndp):
        for t in range(ntp):
            ranks = [int(r) for r in grid[:, d, t]]
            g = _new_group(ranks)
            if rank in ranks:
                _S.pp_group, _S.pp_global_ranks = g, ranks
            if len(ranks) > 1:
                emb = [ranks[0], ranks[-1]]
                pos = [ranks[0]]
                split = pipeline_model_parallel_split_rank
                if split is not None:
                    if ranks[split] not in emb:
                        emb = [ranks[0], ranks[split], ranks[-1]]
                    # independent of the embedding group: the decoder's first
                    # stage may also be the last one (e.g. PP=2, split 1)
                    if ranks[split] not in pos:
                        pos = [ranks[0], ranks[split]]
            else:
                emb, pos = ranks, ranks
            eg = _new_group(emb)
            if rank in emb:
                _S.embedding_group = eg
            if rank in ranks:
                _S.embedding_ranks = emb
            pg = _new_group(pos)
            if rank in pos:
                _S.position_embedding_group = pg
            if rank in ranks:
                _S.position_embedding_ranks = pos
    from . import comm
    for i, g in enumerate(_S.dp_comm_groups[1:]):
        comm.name_group(g, f"dp{i + 1}")
    for g, name in ((_S.dp_group, "dp"), (_S.mp_group, "mp"), (_S.tp_group, "tp"),
                    (_S.pp_group, "pp"), (_S.embedding_group, "emb"),
                    (_S.position_embedding_group, "posemb"), (_S.cp_group, "cp")):
        if g is not None:
            comm.name_group(g, name)


def model_parallel_is_initialized():
    return not (_S.tp_group is None or _S.pp_group is None or _S.dp_group is None)


def _need(group, what):
    if group is None:
        raise RuntimeError(f"{what} group is not initialized")
    return group


def get_model_parallel_group():
    return _need(_S.mp_group, "model parallel")


def get_tensor_model_parallel_group():
    return _need(_S.tp_group, "tensor model parallel")


def get_pipeline_model_parallel_group():
    return _need(_S.pp_group, "pipeline model parallel")


def get_data_parallel_group():
    return _need(_S.dp_group, "data parallel")


def get_data_parallel_comm_groups():
    """[the DP group, extra communicators over the same ranks...]."""
    _need(_S.dp_group, "data parallel")
    return list(_S.dp_comm_groups) or [_S.dp_group]


def get_embedding_group():
    return _need(_S.embedding_group, "embedding")


def get_position_embedding_group():
    return _need(_S.position_embedding_group, "position embedding")


def set_tensor_model_parallel_world_size(world_size):
    _S.tp_world_override = world_size


def set_pipeline_model_parallel_world_size(world_size):
    _S.pp_world_override = world_size


def set_tensor_model_parallel_rank(rank):
    _S.tp_rank_override = rank


def set_pipeline_model_parallel_rank(rank):
    _S.pp_rank_override = rank


def set_pipeline_model_parallel_split_rank(rank):
    _S.pp_split_rank = rank


def _group_size(group):
    if group is None:
        return 1
    return dist.get_world_size(group=group)


def _group_rank(group):
    if group is None:
        return 0
    return dist.get_rank(group=group)


def get_tensor_model_parallel_world_size():
    if _S.tp_world_override is not None:
        return _S.tp_world_override
    return _group_size(_S.tp_group)


def get_pipeline_model_parallel_world_size():
    if _S.pp_world_override is not None:
        return _S.pp_world_override
    return _group_size(_S.pp_group)


def get_tensor_model_parallel_rank():
    if _S.tp_rank_override is not None:
        return _S.tp_rank_override
    return _group_rank(_S.tp_group)


def get_pipeline_model_parallel_rank():
    if _S.pp_rank_override is not None:
        return _S.pp_rank_override
    return _group_rank(_S.pp_group)


def get_pipeline_model_parallel_split_rank():
    return _S.pp_split_rank


def get_data_parallel_world_size():
    return _group_size(_S.dp_group)


def get_data_parallel_rank():
    return _group_rank(_S.dp_group)


def get_context_parallel_group():
    """The ranks sharing one sequence (None when context parallelism is off)."""
    return _S.cp_group


def get_context_parallel_world_size():
    return _S.cp_size if _S.cp_group is not None else 1


def get_context_parallel_rank():
    return _group_rank(_S.cp_group) if _S.cp_group is not None else 0


def get_data_sample_parallel_world_size():
    """Ranks that read different samples: DP / CP."""
    return get_data_parallel_world_size() // get_context_parallel_world_size()


def get_data_sample_parallel_rank():
    return get_data_parallel_rank() // get_context_parallel_world_size()


def get_virtual_pipeline_model_parallel_rank():
    return _S.virtual_pp_rank


def set_virtual_pipeline_model_parallel_rank(rank):
    _S.virtual_pp_rank = rank


def get_virtual_pipeline_model_parallel_world_size():
    return _S.virtual_pp_world_size


def set_virtual_pipeline_model_parallel_world_size(size):
    _S.virtual_pp_world_size = size


def is_pipeline_first_stage(ignore_virtual=False):
    if not ignore_virtual and _S.virtual_pp_world_size is not None \
            and _S.virtual_pp_rank != 0:
        return False
    return get_pipeline_model_parallel_rank() == 0


def is_pipeline_last_stage(ignore_virtual=False):
    if not ignore_virtual and _S.virtual_pp_world_size is not None \
            and _S.virtual_pp_rank != _S.virtual_pp_world_size - 1:
        return False
    return get_pipeline_model_parallel_rank() == get_pipeline_model_parallel_world_size() - 1


def is_rank_in_embedding_group(ignore_virtual=False):
    rank = dist.get_rank()
    if ignore_virtual:
        return rank in _S.embedding_ranks
    if rank not in _S.embedding_ranks:
        return False
    if rank == _S.embedding_ranks[0]:
        return is_pipeline_first_stage(ignore_virtual=False)
    if rank == _S.embedding_ranks[-1]:
        return is_pipeline_last_stage(ignore_virtual=False)
    return True


def is_rank_in_position_embedding_group():
    return dist.get_rank() in _S.position_embedding_ranks


def is_pipeline_stage_before_split(rank=None):
    if get_pipeline_model_parallel_world_size() == 1:
        return True
    rank = get_pipeline_model_parallel_rank() if rank is None else rank
    return _S.pp_split_rank is None or rank < _S.pp_split_rank


def is_pipeline_stage_after_split(rank=None):
    if get_pipeline_model_parallel_world_size() == 1:
        return True
    rank = get_pipeline_model_parallel_rank() if rank is None else rank
    return _S.pp_split_rank is None or rank >= _S.pp_split_rank


def is_pipeline_stage_at_split():
    rank = get_pipeline_model_parallel_rank()
    return is_pipeline_stage_before_split(rank) and is_pipeline_stage_after_split(rank + 1)


def get_tensor_model_parallel_src_rank():
    """Global rank of TP-rank 0 in this rank's TP group."""
    if _S.tp_global_ranks:
        return _S.tp_global_ranks[0]
    rank = dist.get_rank()
    tp = get_tensor_model_parallel_world_size()
    return (rank // tp) * tp


def get_data_parallel_src_rank():
    return _need(_S.dp_global_ranks or None, "data parallel")[0]


def get_pipeline_model_parallel_first_rank():
    return _need(_S.pp_global_ranks or None, "pipeline parallel")[0]


def get_pipeline_model_parallel_last_rank():
    return _need(_S.pp_global_ranks or None, "pipeline parallel")[-1]


def get_pipeline_model_parallel_next_rank():
    ranks = _need(_S.pp_global_ranks or None, "pipeline parallel")
    return ranks[(get_pipeline_model_parallel_rank() + 1) % len(ranks)]


def get_pipeline_model_parallel_prev_rank():
    ranks = _need(_S.pp_global_ranks or None, "pipeline parallel")
    return ranks[(get_pipeline_model_parallel_rank() - 1) % len(ranks)]


def get_global_memory_buffer():
    from .buffers import get_global_memory_buffer as _g
    return _g()


def destroy_model_parallel():
    global _S
    _S = _State()
    from . import buffers
    buffers.reset_global_memory_buffer()
