"""Pipeline point-to-point communication (reference ``megatron/p2p_communication.py``).

Activations ``[s(/tp), b, h]`` move between adjacent stages with batched
``isend/irecv`` on RCCL (xGMI intra-node).  Differences by design:

* No ``torch.cuda.synchronize()`` after every exchange: RCCL
  orders the transfer on its stream; we only ``wait()`` the requests, which
  makes the compute stream wait on the transfer without blocking the host.
* Every exchange goes through ``parallel/comm.py`` (bytes accounting, race
  checker); pure sends stay in flight while the schedule computes and are
  completed before the next exchange / at the end of the schedule.
* Scatter-gather optimisation kept: with TP > 1 and no sequence parallelism
  each TP rank sends only its 1/TP slice and the receiver all-gathers over TP.
* Variable sequence lengths: shapes are exchanged first (int64[3]).
"""
import contextlib
import operator
from functools import reduce

import torch

from .. import comm, state
from ..buffers import make_viewless_tensor
from ..tensor.utils import split_tensor_into_1d_equal_chunks, gather_split_1d_tensor
from ... import global_vars


def _device():
    return torch.cuda.current_device() if torch.cuda.is_available() else "cpu"


_PENDING_SENDS = []  # Work handles of exchanges that only sent (not yet waited)
_DEFER = [0]  # > 0 inside a pipeline schedule: pure sends may stay in flight


@contextlib.contextmanager
def deferred_sends():
    """Scope (the pipeline schedules) in which pure sends are left in flight;
    every one of them is completed when the scope ends.  Outside it (inference,
    evaluation, tools) a send is completed before ``send_*`` returns, so a rank
    can never exit with its last activation still queued."""
    _DEFER[0] += 1
    try:
        yield
    finally:
        _DEFER[0] -= 1
        wait_pending_sends()


def wait_pending_sends():
    """Complete every deferred pure-send exchange (called before the next
    exchange and at the end of each schedule)."""
    while _PENDING_SENDS:
        _PENDING_SENDS.pop(0).wait()


def _p2p(ops):
    """Post ``ops`` [(kind, tensor, peer)] through the collective layer.

    An exchange that receives is waited at once (its consumer runs next); one
    that only sends is left in flight while the schedule computes and is
    completed before the next exchange (RCCL keeps the send buffers alive;
    the buffers are passed as detached aliases, so the schedules' pseudo-free
    of a sent output tensor cannot swap them out from under the transfer)."""
    wait_pending_sends()
    ops = [(k, t.detach() if k == "send" else t, peer) for k, t, peer in
           (o for o in ops if o is not None)]
    if not ops:
        return
    group = state.get_pipeline_model_parallel_group()
    if _DEFER[0] > 0 and all(k == "send" for k, _, _ in ops):
        h = comm.p2p(ops, group=group, async_op=True)
        if h is not None:
            _PENDING_SENDS.append(h)
    else:
        comm.p2p(ops, group=group)


def _communicate_shapes(tensor_send_next, tensor_send_prev, recv_prev, recv_next):
    dev = _device()
    recv_prev_shape = torch.empty(3, dtype=torch.int64, device=dev) if recv_prev else None
    recv_next_shape = torch.empty(3, dtype=torch.int64, device=dev) if recv_next else None
    send_next_shape = torch.tensor(tensor_send_next.size(), dtype=torch.int64, device=dev) \
        if tensor_send_next is not None else None
    send_prev_shape = torch.tensor(tensor_send_prev.size(), dtype=torch.int64, device=dev) \
        if tensor_send_prev is not None else None
    prev_r = state.get_pipeline_model_parallel_prev_rank()
    next_r = state.get_pipeline_model_parallel_next_rank()
    ops = [
        ("send", send_prev_shape, prev_r) if send_prev_shape is not None else None,
        ("recv", recv_prev_shape, prev_r) if recv_prev_shape is not None else None,
        ("send", send_next_shape, next_r) if send_next_shape is not None else None,
        ("recv", recv_next_shape, next_r) if recv_next_shape is not None else None,
    ]
    _p2p(ops)
    return ([int(x) for x in recv_prev_shape.tolist()] if recv_prev else None,
            [int(x) for x in recv_next_shape.tolist()] if recv_next else None)


def _communicate(tensor_send_next, tensor_send_prev, recv_prev, recv_next, tensor_shape,
                 dtype_=None):
    args = global_vars.get_args()
    if args.variable_seq_lengths:
        rp_shape, rn_shape = _communicate_shapes(tensor_send_next, tensor_send_prev, recv_prev,
                                                 recv_next)
    else:
        rp_shape = rn_shape = list(tensor_shape)
    tp = state.get_tensor_model_parallel_world_size()
    scatter_gather = (args.scatter_gather_tensors_in_pipeline and not args.sequence_parallel
                      and tp > 1)

    def flat_shape(shape):
        n = reduce(operator.mul, shape, 1)
        return (n // tp,) if scatter_gather else tuple(shape)

    dtype = dtype_ or (args.params_dtype if (args.fp16 or args.bf16) else torch.float)
    dev = _device()
    recv_prev_t = torch.empty(flat_shape(rp_shape), dtype=dtype, device=dev,
                              requires_grad=True) if recv_prev else None
    recv_next_t = torch.empty(flat_shape(rn_shape), dtype=dtype, device=dev,
                              requires_grad=True) if recv_next else None
    if scatter_gather:
        if tensor_send_next is not None:
            tensor_send_next = split_tensor_into_1d_equal_chunks(tensor_send_next)
        if tensor_send_prev is not None:
            tensor_send_prev = split_tensor_into_1d_equal_chunks(tensor_send_prev)
    prev_r = state.get_pipeline_model_parallel_prev_rank()
    next_r = state.get_pipeline_model_parallel_next_rank()
    # Post order: activations (forward direction) before gradients (backward
    # direction).  RCCL/NCCL match the point-to-point operations of one peer
    # pair in posting order; with PP = 2 both messages of a combined
    # send-forward/send-backward go to the SAME peer, so this order is what
    # keeps "activation" matched with "activation" on the other side (the
    # reference's order swapped them, which is why it forbade interleaving at
    # PP = 2, megatron/arguments.py:117-120).
    ops = []
    if tensor_send_next is not None:
        ops.append(("send", tensor_send_next.contiguous(), next_r))
    if recv_prev_t is not None:
        ops.append(("recv", recv_prev_t, prev_r))
    if tensor_send_prev is not None:
        ops.append(("send", tensor_send_prev.contiguous(), prev_r))
    if recv_next_t is not None:
        ops.append(("recv", recv_next_t, next_r))
    _p2p(ops)
    if scatter_gather:
        if recv_prev:
            recv_prev_t = gather_split_1d_tensor(recv_prev_t).view(rp_shape).requires_grad_()
            recv_prev_t = make_viewless_tensor(recv_prev_t, requires_grad=True, keep_graph=False)
        if recv_next:
            recv_next_t = gather_split_1d_tensor(recv_next_t).view(rn_shape).requires_grad_()
            recv_next_t = make_viewless_tensor(recv_next_t, requires_grad=True, keep_graph=False)
    return recv_prev_t, recv_next_t


def _timed(timers, name):
    class _Ctx:
        def __enter__(self_inner):
            if timers is not None:
                timers(name, log_level=2).start()

        def __exit__(self_inner, *a):
            if timers is not None:
                timers(name).stop()
    return _Ctx()


def recv_forward(tensor_shape=None, dtype_=None, timers=None):
    if state.is_pipeline_first_stage():
        return None
    with _timed(timers, "forward-recv"):
        t, _ = _communicate(None, None, True, False, tensor_shape, dtype_)
    return t


def recv_backward(tensor_shape=None, timers=None):
    if state.is_pipeline_last_stage():
        return None
    with _timed(timers, "backward-recv"):
        _, t = _communicate(None, None, False, True, tensor_shape)
    return t


def send_forward(output_tensor, tensor_shape=None, dtype_=None, timers=None):
    if state.is_pipeline_last_stage():
        return
    with _timed(timers, "forward-send"):
        _communicate(output_tensor, None, False, False, tensor_shape, dtype_)


def send_backward(input_tensor_grad, tensor_shape=None, timers=None):
    if state.is_pipeline_first_stage():
        return
    with _timed(timers, "backward-send"):
        _communicate(None, input_tensor_grad, False, False, tensor_shape)


def send_forward_recv_backward(output_tensor, tensor_shape=None, timers=None):
    if state.is_pipeline_last_stage():
        return None
    with _timed(timers, "forward-send-backward-recv"):
        _, g = _communicate(output_tensor, None, False, True, tensor_shape)
    return g


def send_backward_recv_forward(input_tensor_grad, tensor_shape=None, timers=None):
    if state.is_pipeline_first_stage():
        return None
    with _timed(timers, "backward-send-forward-recv"):
        t, _ = _communicate(None, input_tensor_grad, True, False, tensor_shape)
    return t


def send_forward_recv_forward(output_tensor, recv_prev, tensor_shape=None, timers=None):
    with _timed(timers, "forward-send-forward-recv"):
        t, _ = _communicate(output_tensor, None, recv_prev, False, tensor_shape)
    return t


def send_backward_recv_backward(input_tensor_grad, recv_next, tensor_shape=None, timers=None):
    with _timed(timers, "backward-send-backward-recv"):
        _, g = _communicate(None, input_tensor_grad, False, recv_next, tensor_shape)
    return g


def send_forward_backward_recv_forward_backward(output_tensor, input_tensor_grad, recv_prev,
                                                recv_next, tensor_shape=None, timers=None):
    with _timed(timers, "forward-backward-send-forward-backward-recv"):
        t, g = _communicate(output_tensor, input_tensor_grad, recv_prev, recv_next, tensor_shape)
    return t, g
