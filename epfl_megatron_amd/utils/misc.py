"""General utilities (reference ``megatron/utils.py``)."""
import sys

import torch
import torch.distributed as dist
from torch.nn.parallel import DistributedDataParallel as torchDDP

from ..parallel import state


def unwrap_model(model, module_instances=None):
    from ..parallel.ddp import DistributedDataParallel as LocalDDP
    from ..models.module import Float16Module
    module_instances = module_instances or (torchDDP, LocalDDP, Float16Module)
    single = not isinstance(model, list)
    models = [model] if single else model
    out = []
    for m in models:
        while isinstance(m, module_instances):
            m = m.module
        out.append(m)
    return out[0] if single else out


def calc_params_l2_norm(model):
    """L2 norm of non-duplicated, non-shared params, summed over model parallel."""
    from ..parallel.tensor import param_is_not_tensor_parallel_duplicate
    from ..models.module import param_is_not_shared
    models = model if isinstance(model, list) else [model]
    sq = None
    for m in models:
        if hasattr(m, "wait_param_sync"):  # dist-opt all-gather may be in flight
            m.wait_param_sync()
        for p in m.parameters():
            if param_is_not_shared(p) and param_is_not_tensor_parallel_duplicate(p):
                v = p.detach().float().pow(2).sum()
                sq = v if sq is None else sq + v
    if sq is None:
        sq = torch.zeros((), device=torch.cuda.current_device() if torch.cuda.is_available() else "cpu")
    sq = sq.reshape(1)
    if dist.is_initialized():
        from ..parallel import comm  # noqa: PLC0415
        comm.all_reduce(sq, group=state.get_model_parallel_group())
    return sq.item() ** 0.5


def average_losses_across_data_parallel_group(losses):
    """Logging-only DP average (one fused collective, averaged inside it)."""
    averaged = torch.cat([l.clone().detach().view(1) for l in losses])
    if dist.is_initialized() and state.get_data_parallel_world_size() > 1:
        from ..parallel import comm
        comm.all_reduce(averaged, group=state.get_data_parallel_group(), op="avg")
    return averaged


def report_memory(name):
    if not torch.cuda.is_available():
        return
    mb = 1024.0 * 1024.0
    s = (f"[{name}] memory (MB) | allocated: {torch.cuda.memory_allocated() / mb} | "
         f"max allocated: {torch.cuda.max_memory_allocated() / mb} | "
         f"reserved: {torch.cuda.memory_reserved() / mb} | "
         f"max reserved: {torch.cuda.max_memory_reserved() / mb}")
    if state.get_data_parallel_rank() == 0:
        print(f"[Rank {dist.get_rank() if dist.is_initialized() else 0}] {s}", flush=True)


def doc_bounds(data, eod_token):
    """Document bounds of packed sequences: int32 ``[2, b, s]`` with, per
    position, the first position of its document and one past its last.
    A document ends WITH its EOD token (the EOD row still sees its own
    document; the row after it starts a new one), as in the reference's
    mask loop (``megatron/utils.py:137-194``)."""
    b, s = data.shape
    pos = torch.arange(s, device=data.device)
    is_eod = data == eod_token
    starts = torch.zeros((b, s), dtype=torch.long, device=data.device)
    starts[:, 1:] = torch.where(is_eod[:, :-1], pos[1:], 0)
    start = torch.cummax(starts, dim=1).values
    ends = torch.where(is_eod, pos + 1, s)
    end = torch.flip(torch.cummin(torch.flip(ends, [1]), dim=1).values, [1])
    return torch.stack([start, end]).to(torch.int32).contiguous()


def get_ltor_masks_and_position_ids(data, eod_token, reset_position_ids, reset_attention_mask,
                                    eod_mask_loss, flash_doc_bounds=False):
    """Causal mask (True = masked) ``[1 or b, 1, s, s]``, loss mask and position ids.

    With reset flags, positions / attention restart after every EOD token of
    each sample (reference ``megatron/utils.py:137-194``), computed from
    :func:`doc_bounds` without a per-EOD loop.  ``flash_doc_bounds``: with
    ``reset_attention_mask``, return the int32 ``[2, b, s]`` document bounds
    in place of the dense mask (the flash-attention kernels mask documents
    from them; no ``b x s x s`` tensor is built)."""
    b, s = data.size()
    loss_mask = torch.ones(data.size(), dtype=torch.float, device=data.device)
    if eod_mask_loss:
        loss_mask[data == eod_token] = 0.0
    position_ids = torch.arange(s, dtype=torch.long, device=data.device)
    position_ids = position_ids.unsqueeze(0).expand_as(data)
    bounds = doc_bounds(data, eod_token) if (reset_position_ids or reset_attention_mask) else None
    if reset_position_ids:
        position_ids = (position_ids - bounds[0].long()).contiguous()
    if reset_attention_mask and flash_doc_bounds:
        return bounds, loss_mask, position_ids
    i = torch.arange(s, device=data.device)[:, None]
    j = torch.arange(s, device=data.device)[None, :]
    masked = (j > i)[None]  # [1, s, s]
    if reset_attention_mask:
        masked = masked | (j[None] < bounds[0].long()[:, :, None])  # [b, s, s]
    return masked.unsqueeze(1), loss_mask, position_ids


def _rank():
    return dist.get_rank() if dist.is_initialized() else 0


def print_rank_0(message):
    if _rank() == 0:
        print(message, flush=True)


def is_last_rank():
    if not dist.is_initialized():
        return True
    return dist.get_rank() == dist.get_world_size() - 1


def print_rank_last(message):
    if is_last_rank():
        print(message, flush=True)


def print_all_nodes(message):
    import os
    lws = int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
    if _rank() % max(lws, 1) == lws - 1 or not dist.is_initialized():
        print(message, flush=True)


def check_adlr_autoresume_termination(iteration, model, optimizer, opt_param_scheduler):
    from .. import global_vars
    from ..checkpointing import save_checkpoint
    autoresume = global_vars.get_adlr_autoresume()
    if dist.is_initialized():
        dist.barrier()
    if autoresume is not None and autoresume.termination_requested():
        save_checkpoint(iteration, model, optimizer, opt_param_scheduler)
        print_rank_0(">>> autoresume termination request found!")
        if _rank() == 0:
            autoresume.request_resume()
        print_rank_0(">>> training terminated. Returning")
        sys.exit(0)
