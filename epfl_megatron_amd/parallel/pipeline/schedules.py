"""Microbatch schedules: no pipelining, 1F1B, interleaved 1F1B.

Schedule math follows the reference (``megatron/schedules.py``; SURVEY §2.7
"1F1B" / "Interleaved 1F1B"): 1F1B warms up with ``pp - rank - 1`` forwards;
interleaved uses ``(pp - rank - 1) * 2 + (chunks - 1) * pp`` warm-up
microbatches and maps microbatch k to chunk ``(k mod (pp*chunks)) // pp``
(reversed in backward).  Pipeline outputs are "pseudo-freed" after being sent
(only the autograd graph is kept).  Interleaving at PP = 2 is permitted with
``--allow_interleaved_pp2`` (the math holds; the reference forbade it).

DP gradient reduction overlaps with backward: the DDP wrapper launches bucket
collectives during the LAST backward of each model chunk only (gradient
accumulation across the earlier microbatches stays local).
"""
import functools
import contextlib

import torch
from torch.autograd.variable import Variable

from .. import state
from ..buffers import make_viewless_tensor
from ... import global_vars
from . import p2p
from ...models.enums import ModelType
from ...utils.trace import trace_range, tracing


def get_forward_backward_func():
    args = global_vars.get_args()
    if state.get_pipeline_model_parallel_world_size() > 1:
        if args.virtual_pipeline_model_parallel_size is not None:
            return forward_backward_pipelining_with_interleaving
        return forward_backward_pipelining_without_interleaving
    return forward_backward_no_pipelining


def deallocate_output_tensor(out):
    """Keep only the autograd graph of a sent pipeline output (frees activation memory)."""
    if out is None:
        return
    if out._base is not None:
        raise AssertionError("counter-productive to free a view of another tensor.")
    out.data = torch.empty((1,), device=out.device, dtype=out.dtype)


def custom_backward(output, grad_output):
    """Backward that skips the output/grad shape check (output was pseudo-freed)."""
    if output.numel() != 1 and grad_output is None:
        raise AssertionError("implicit grad requires scalar output.")
    if grad_output is None:
        grad_output = torch.ones_like(output, memory_format=torch.preserve_format)
    Variable._execution_engine.run_backward(
        tensors=(output,), grad_tensors=(grad_output,), keep_graph=False, create_graph=False,
        inputs=tuple(), allow_unreachable=True, accumulate_grad=True)


def _unwrap(model):
    from ...utils.misc import unwrap_model
    return unwrap_model(model)


def forward_step(forward_step_func, data_iterator, model, input_tensor, forward_data_store,
                 timers, collect_non_loss_data=False):
    if tracing():
        with trace_range("fwd-microbatch"):
            return _forward_step(forward_step_func, data_iterator, model, input_tensor,
                                 forward_data_store, timers, collect_non_loss_data)
    return _forward_step(forward_step_func, data_iterator, model, input_tensor,
                         forward_data_store, timers, collect_non_loss_data)


def _forward_step(forward_step_func, data_iterator, model, input_tensor, forward_data_store,
                  timers, collect_non_loss_data=False):
    if timers is not None:
        timers("forward-compute", log_level=2).start()
    unwrapped = _unwrap(model)
    unwrap_output = False
    if not isinstance(input_tensor, list):
        input_tensor = [input_tensor]
        unwrap_output = True
    unwrapped.set_input_tensor(input_tensor)
    output_tensor, loss_func = forward_step_func(data_iterator, model)
    if state.is_pipeline_last_stage():
        if not collect_non_loss_data:
            output_tensor = loss_func(output_tensor)
            loss, loss_reduced = output_tensor
            output_tensor = loss / global_vars.get_num_microbatches()
            forward_data_store.append(loss_reduced)
        else:
            forward_data_store.append(loss_func(output_tensor, non_loss_data=True))
    if timers is not None:
        timers("forward-compute").stop()
    if unwrap_output:
        return output_tensor
    return [output_tensor]


def backward_step(optimizer, input_tensor, output_tensor, output_tensor_grad, timers):
    if tracing():
        with trace_range("bwd-microbatch"):
            return _backward_step(optimizer, input_tensor, output_tensor, output_tensor_grad,
                                  timers)
    return _backward_step(optimizer, input_tensor, output_tensor, output_tensor_grad, timers)


def _backward_step(optimizer, input_tensor, output_tensor, output_tensor_grad, timers):
    if timers is not None:
        timers("backward-compute", log_level=2).start()
    unwrap_input = False
    if not isinstance(input_tensor, list):
        input_tensor, unwrap_input = [input_tensor], True
    for t in input_tensor:
        if t is not None:
            t.retain_grad()
    if not isinstance(output_tensor, list):
        output_tensor = [output_tensor]
    if not isinstance(output_tensor_grad, list):
        output_tensor_grad = [output_tensor_grad]
    if output_tensor_grad[0] is None:
        output_tensor[0] = optimizer.scale_loss(output_tensor[0])
    custom_backward(output_tensor[0], output_tensor_grad[0])
    input_tensor_grad = [t.grad if t is not None else None for t in input_tensor]
    if timers is not None:
        timers("backward-compute").stop()
    return input_tensor_grad[0] if unwrap_input else input_tensor_grad


@contextlib.contextmanager
def _grad_sync(model, enabled):
    setter = getattr(model, "set_grad_sync", None)
    if setter is None:
        yield
        return
    setter(enabled)
    try:
        yield
    finally:
        setter(True)


def forward_backward_no_pipelining(forward_step_func, data_iterator, model, optimizer, timers,
                                   forward_only, collect_non_loss_data=False):
    if isinstance(model, list):
        if len(model) != 1:
            raise AssertionError("non-pipeline-parallel schedule does not support model chunking")
        model = model[0]
    store = []
    input_tensor, output_tensor_grad = None, None
    m = global_vars.get_num_microbatches()
    for i in range(m):
        last = i == m - 1
        with _grad_sync(model, last):
            out = forward_step(forward_step_func, data_iterator, model, input_tensor, store,
                               timers, collect_non_loss_data)
            if not forward_only:
                backward_step(optimizer, input_tensor, out, output_tensor_grad, timers)
    return store


def get_tensor_shapes(rank, model_type):
    args = global_vars.get_args()
    seq = args.seq_length // state.get_context_parallel_world_size()
    if args.sequence_parallel:
        seq = seq // state.get_tensor_model_parallel_world_size()
    if model_type == ModelType.encoder_and_decoder:
        dec = args.decoder_seq_length
        if args.sequence_parallel:
            dec = dec // state.get_tensor_model_parallel_world_size()
        if state.is_pipeline_stage_before_split(rank):
            return [(seq, args.micro_batch_size, args.hidden_size)]
        return [(dec, args.micro_batch_size, args.hidden_size),
                (seq, args.micro_batch_size, args.hidden_size)]
    return [(seq, args.micro_batch_size, args.hidden_size)]


def _recv_forward(shapes, timers):
    return [p2p.recv_forward(s, timers=timers) if s is not None else None for s in shapes]


def _recv_backward(shapes, timers):
    return [p2p.recv_backward(s, timers=timers) if s is not None else None for s in shapes]


def _send_forward(outs, shapes, timers):
    if not isinstance(outs, list):
        outs = [outs]
    for o, s in zip(outs, shapes):
        if s is not None:
            p2p.send_forward(o, s, timers=timers)


def _send_backward(grads, shapes, timers):
    if not isinstance(grads, list):
        grads = [grads]
    for g, s in zip(grads, shapes):
        if s is not None:
            p2p.send_backward(g, s, timers=timers)


def _send_forward_recv_backward(outs, shapes, timers):
    if not isinstance(outs, list):
        outs = [outs]
    return [p2p.send_forward_recv_backward(o, s, timers=timers) if s is not None else None
            for o, s in zip(outs, shapes)]


def _send_backward_recv_forward(grads, shapes, timers):
    if not isinstance(grads, list):
        grads = [grads]
    return [p2p.send_backward_recv_forward(g, s, timers=timers) if s is not None else None
            for g, s in zip(grads, shapes)]


def _deferred_sends(fn):
    """Run a pipelined schedule with its pure sends left in flight between
    exchanges (``p2p.deferred_sends``)."""
    @functools.wraps(fn)
    def wrapper(*a, **k):
        with p2p.deferred_sends():
            return fn(*a, **k)
    return wrapper


@_deferred_sends
def forward_backward_pipelining_without_interleaving(forward_step_func, data_iterator, model,
                                                     optimizer, timers, forward_only,
                                                     collect_non_loss_data=False):
    """Non-interleaved 1F1B."""
    args = global_vars.get_args()
    if isinstance(model, list):
        if len(model) != 1:
            raise AssertionError("non-interleaved pipeline does not support model chunking")
        model = model[0]
    m = global_vars.get_num_microbatches()
    pp = state.get_pipeline_model_parallel_world_size()
    rank = state.get_pipeline_model_parallel_rank()
    warmup = min(pp - rank - 1, m)
    steady = m - warmup
    model_type = _unwrap(model).model_type if hasattr(_unwrap(model), "model_type") \
        else ModelType.encoder_or_decoder
    recv_shapes = get_tensor_shapes(rank - 1, model_type)
    send_shapes = get_tensor_shapes(rank, model_type)
    inputs, outputs, store = [], [], []
    backward_done = 0

    def run_backward(inp, out, grad):
        nonlocal backward_done
        backward_done += 1
        with _grad_sync(model, backward_done == m):
            return backward_step(optimizer, inp, out, grad, timers)

    with _grad_sync(model, False):
        for _ in range(warmup):
            inp = _recv_forward(recv_shapes, timers)
            out = forward_step(forward_step_func, data_iterator, model, inp, store, timers,
                               collect_non_loss_data)
            _send_forward(out, send_shapes, timers)
            if not forward_only:
                inputs.append(inp)
                outputs.append(out)
                deallocate_output_tensor(out[0])
    inp = _recv_forward(recv_shapes, timers) if steady > 0 else None
    for i in range(steady):
        last = i == steady - 1
        out = forward_step(forward_step_func, data_iterator, model, inp, store, timers,
                           collect_non_loss_data)
        if forward_only:
            _send_forward(out, send_shapes, timers)
            if not last:
                inp = _recv_forward(recv_shapes, timers)
            continue
        out_grad = _send_forward_recv_backward(out, send_shapes, timers)
        inputs.append(inp)
        outputs.append(out)
        deallocate_output_tensor(out[0])
        inp, out = inputs.pop(0), outputs.pop(0)
        in_grad = run_backward(inp, out, out_grad)
        if last:
            inp = None
            _send_backward(in_grad, recv_shapes, timers)
        else:
            inp = _send_backward_recv_forward(in_grad, recv_shapes, timers)
    if not forward_only:
        for _ in range(warmup):
            inp, out = inputs.pop(0), outputs.pop(0)
            out_grad = _recv_backward(send_shapes, timers)
            in_grad = run_backward(inp, out, out_grad)
            _send_backward(in_grad, recv_shapes, timers)
    p2p.wait_pending_sends()
    return store


@_deferred_sends
def forward_backward_pipelining_with_interleaving(forward_step_func, data_iterator, model,
                                                  optimizer, timers, forward_only,
                                                  collect_non_loss_data=False):
    """Interleaved 1F1B over ``len(model)`` virtual stages per rank."""
    args = global_vars.get_args()
    chunks = len(model)
    inputs = [[] for _ in range(chunks)]
    outputs = [[] for _ in range(chunks)]
    out_grads = [[] for _ in range(chunks)]
    store = []
    pp = state.get_pipeline_model_parallel_world_size()
    rank = state.get_pipeline_model_parallel_rank()
    m = global_vars.get_num_microbatches()
    if m % pp != 0:
        raise RuntimeError(f"number of microbatches ({m}) is not divisible by pipeline-model-"
                           f"parallel size ({pp}) when using interleaved schedule")
    seq = args.seq_length // state.get_context_parallel_world_size()
    if args.sequence_parallel:
        seq //= state.get_tensor_model_parallel_world_size()
    shape = (seq, args.micro_batch_size, args.hidden_size)
    total = m * chunks
    all_warmup = False
    if forward_only:
        warmup = total
    elif m == pp:
        warmup, all_warmup = total, True
    else:
        warmup = min((pp - rank - 1) * 2 + (chunks - 1) * pp, total)
    remaining = total - warmup
    backward_counts = [0] * chunks

    def chunk_id(k, forward):
        cid = (k % (pp * chunks)) // pp
        return cid if forward else chunks - cid - 1

    def fwd(k):
        cid = chunk_id(k, True)
        state.set_virtual_pipeline_model_parallel_rank(cid)
        if state.is_pipeline_first_stage() and len(inputs[cid]) == len(outputs[cid]):
            inputs[cid].append(None)
        inp = inputs[cid][-1]
        with _grad_sync(model[cid], False):
            out = forward_step(forward_step_func, data_iterator[cid], model[cid], inp, store,
                               timers, collect_non_loss_data)
        outputs[cid].append(out)
        if forward_only:
            inputs[cid].pop()
            outputs[cid].pop()
        return out

    def bwd(k):
        cid = chunk_id(k, False)
        state.set_virtual_pipeline_model_parallel_rank(cid)
        if state.is_pipeline_last_stage() and len(out_grads[cid]) == 0:
            out_grads[cid].append(None)
        inp = inputs[cid].pop(0)
        out = outputs[cid].pop(0)
        g = out_grads[cid].pop(0)
        backward_counts[cid] += 1
        with _grad_sync(model[cid], backward_counts[cid] == m):
            return backward_step(optimizer, inp, out, g, timers)

    state.set_virtual_pipeline_model_parallel_rank(0)
    inputs[0].append(p2p.recv_forward(shape, timers=timers))
    for k in range(warmup):
        out = fwd(k)
        nxt = chunk_id(k + 1, True)
        recv_prev = True
        if state.is_pipeline_first_stage(ignore_virtual=True) and nxt == 0:
            recv_prev = False
        if k == total - 1:
            recv_prev = False
        if state.is_pipeline_last_stage():
            out = None
        if k == warmup - 1 and not forward_only and not all_warmup:
            recv_next = not state.is_pipeline_last_stage(ignore_virtual=True)
            inp, g = p2p.send_forward_backward_recv_forward_backward(
                out, None, recv_prev, recv_next, shape, timers=timers)
            out_grads[chunks - 1].append(g)
        else:
            inp = p2p.send_forward_recv_forward(out, recv_prev, shape, timers=timers)
        inputs[nxt].append(inp)
        if out is not None:
            deallocate_output_tensor(out)
    for k in range(remaining):
        fk = k + warmup
        out = fwd(fk)
        in_grad = bwd(k)
        state.set_virtual_pipeline_model_parallel_rank(chunk_id(fk, True))
        if state.is_pipeline_last_stage():
            out = None
        state.set_virtual_pipeline_model_parallel_rank(chunk_id(k, False))
        if state.is_pipeline_first_stage():
            in_grad = None
        recv_prev = True
        if state.is_pipeline_first_stage(ignore_virtual=True):
            nf = chunk_id(fk - (pp - 1), True)
            if nf == chunks - 1:
                recv_prev = False
            nf += 1
        else:
            nf = chunk_id(fk + 1, True)
        recv_next = True
        if state.is_pipeline_last_stage(ignore_virtual=True):
            nb = chunk_id(k - (pp - 1), False)
            if nb == 0:
                recv_next = False
            nb -= 1
        else:
            nb = chunk_id(k + 1, False)
        if k == remaining - 1:
            recv_prev = False
        inp, g = p2p.send_forward_backward_recv_forward_backward(
            out, in_grad, recv_prev, recv_next, shape, timers=timers)
        if out is not None:
            deallocate_output_tensor(out)
        if recv_prev:
            inputs[nf].append(inp)
        if recv_next:
            out_grads[nb].append(g)
    if not forward_only:
        if all_warmup:
            out_grads[chunks - 1].append(p2p.recv_backward(shape, timers=timers))
        for k in range(remaining, total):
            in_grad = bwd(k)
            nb = chunk_id(k + 1, False)
            recv_next = True
            if state.is_pipeline_last_stage(ignore_virtual=True) and nb == chunks - 1:
                recv_next = False
            if k == total - 1:
                recv_next = False
            out_grads[nb].append(p2p.send_backward_recv_backward(in_grad, recv_next, shape,
                                                                 timers=timers))
    p2p.wait_pending_sends()
    state.set_virtual_pipeline_model_parallel_rank(0)
    return store
