"""Collectives used by the inference loop (reference ``megatron/text_generation/communication.py``).

All helpers run on the default device of the backend (HIP for RCCL, CPU for
gloo) so the same serving code runs in CPU tests.  Point-to-point transfers
between pipeline stages use blocking ``send``/``recv`` of pre-shaped buffers;
broadcasts "from the last stage" use the embedding group's peer-free route:
a ``broadcast`` over the whole world rooted at the last pipeline rank of this
rank's pipeline (the reference did the same, :59-110).
"""
import torch
import torch.distributed as dist

from ..parallel import comm, state


def device():
    if dist.is_initialized() and dist.get_backend() == "gloo":
        return torch.device("cpu")
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
        else torch.device("cpu")


def recv_from_prev_pipeline_rank_(recv_buffer=None):
    """Receive into ``recv_buffer`` from the previous stage (no-op on the first)."""
    if not state.is_pipeline_first_stage():
        if recv_buffer is None:
            raise AssertionError("a receive buffer is required on non-first stages")
        dist.recv(recv_buffer, state.get_pipeline_model_parallel_prev_rank())


def send_to_next_pipeline_rank(tensor=None):
    if not state.is_pipeline_last_stage():
        if tensor is None:
            raise AssertionError("nothing to send to the next stage")
        dist.send(tensor.contiguous(), state.get_pipeline_model_parallel_next_rank())


def _is_cuda_contiguous(t):
    return t.is_contiguous() and t.device == device()


def broadcast_from_last_pipeline_stage(size, dtype, tensor=None):
    """Broadcast ``tensor`` (given on the last stage) to every rank of its pipeline."""
    if state.is_pipeline_last_stage():
        if not _is_cuda_contiguous(tensor):
            raise AssertionError("tensor must be contiguous on the communication device")
    else:
        tensor = torch.empty(size, dtype=dtype, device=device())
    if state.get_pipeline_model_parallel_world_size() > 1:
        comm.broadcast(tensor, state.get_pipeline_model_parallel_last_rank(),
                       group=state.get_pipeline_model_parallel_group())
    return tensor


def broadcast_from_last_to_first_pipeline_stage(size, dtype, tensor=None):
    """Last stage -> first stage (other stages return None)."""
    first, last = state.is_pipeline_first_stage(), state.is_pipeline_last_stage()
    if first and last:
        return tensor
    if not (first or last):
        return None
    if last:
        if not _is_cuda_contiguous(tensor):
            raise AssertionError("tensor must be contiguous on the communication device")
    else:
        tensor = torch.empty(size, dtype=dtype, device=device())
    comm.broadcast(tensor, state.get_pipeline_model_parallel_last_rank(),
                   group=state.get_embedding_group())
    return tensor


def copy_from_last_to_first_pipeline_stage(size, dtype, tensor=None):
    """In-place copy of ``tensor`` from the last stage into the first stage's tensor."""
    first, last = state.is_pipeline_first_stage(), state.is_pipeline_last_stage()
    if (first and last) or not (first or last):
        return
    if tensor is None:
        raise AssertionError("tensor required on the first and last stages")
    buf = tensor if tensor.is_contiguous() else torch.empty(size, dtype=dtype, device=device())
    if last and buf is not tensor:
        buf.copy_(tensor)
    comm.broadcast(buf, state.get_pipeline_model_parallel_last_rank(),
                   group=state.get_embedding_group())
    if first and buf is not tensor:
        tensor.copy_(buf)


def broadcast_tensor(size, dtype, tensor=None, rank=0):
    """World broadcast of a tensor that exists on ``rank`` only."""
    if dist.get_rank() == rank:
        if not _is_cuda_contiguous(tensor):
            raise AssertionError("tensor must be contiguous on the communication device")
    else:
        tensor = torch.empty(size, dtype=dtype, device=device())
    comm.broadcast(tensor, rank)
    return tensor


def broadcast_list(size, dtype, list_values=None, rank=0):
    t = torch.tensor(list_values, dtype=dtype, device=device()) if dist.get_rank() == rank \
        else None
    return broadcast_tensor(size, dtype, tensor=t, rank=rank)


def broadcast_int_list(size, int_list=None, rank=0):
    return broadcast_list(size, torch.int64, list_values=int_list, rank=rank)


def broadcast_float_list(size, float_list=None, rank=0):
    return broadcast_list(size, torch.float32, list_values=float_list, rank=rank)
