"""RNG streams and RNG-consistent activation checkpointing.

Contract (reference ``megatron/core/tensor_parallel/random.py:64-252``):
the default device RNG is identical across TP ranks (seeded from the global
seed + 100*pp_rank), while the ``model-parallel-rng`` stream differs per TP
rank (``seed + 2718 + tp_rank``) and is used for TP-sharded weight init and
dropout inside TP regions.  ``checkpoint`` saves/restores the CPU, device and
tracker states so recomputation replays the exact dropout masks.
"""
import contextlib

import torch
from torch.utils.checkpoint import detach_variable

from .. import state
from ..buffers import safely_set_viewless_tensor_data
from .utils import gather_split_1d_tensor, split_tensor_into_1d_equal_chunks

_MODEL_PARALLEL_RNG_TRACKER_NAME = "model-parallel-rng"


def _device_available():
    return torch.cuda.is_available()


def _get_device_rng_state():
    if _device_available():
        return torch.cuda.get_rng_state()
    return torch.get_rng_state()


def _set_device_rng_state(new_state):
    if _device_available():
        torch.cuda.set_rng_state(new_state)
    else:
        torch.set_rng_state(new_state)


def _manual_seed_device(seed):
    if _device_available():
        torch.cuda.manual_seed(seed)
    else:
        torch.manual_seed(seed)


class CudaRNGStatesTracker:
    """Named device-RNG states; ``fork(name)`` swaps one in for a region."""

    def __init__(self):
        self.states_ = {}
        self.seeds_ = set()

    def reset(self):
        self.states_ = {}
        self.seeds_ = set()

    def get_states(self):
        return dict(self.states_)

    def set_states(self, states):
        self.states_ = dict(states)

    def add(self, name, seed):
        if seed in self.seeds_:
            raise Exception(f"seed {seed} already exists")
        if name in self.states_:
            raise Exception(f"cuda rng state {name} already exists")
        self.seeds_.add(seed)
        saved = _get_device_rng_state()
        _manual_seed_device(seed)
        self.states_[name] = _get_device_rng_state()
        _set_device_rng_state(saved)

    @contextlib.contextmanager
    def fork(self, name=_MODEL_PARALLEL_RNG_TRACKER_NAME):
        if name not in self.states_:
            raise Exception(f"cuda rng state {name} is not added")
        saved = _get_device_rng_state()
        _set_device_rng_state(self.states_[name])
        try:
            yield
        finally:
            self.states_[name] = _get_device_rng_state()
            _set_device_rng_state(saved)


_CUDA_RNG_STATE_TRACKER = CudaRNGStatesTracker()


def get_cuda_rng_tracker():
    return _CUDA_RNG_STATE_TRACKER


def model_parallel_cuda_manual_seed(seed):
    """Default stream = ``seed`` (same on all TP ranks); TP stream = seed+2718+tp_rank."""
    tp_seed = seed + 2718 + state.get_tensor_model_parallel_rank()
    _CUDA_RNG_STATE_TRACKER.reset()
    _manual_seed_device(seed)
    _CUDA_RNG_STATE_TRACKER.add(_MODEL_PARALLEL_RNG_TRACKER_NAME, tp_seed)


class CheckpointFunction(torch.autograd.Function):
    """Drop activations in forward; recompute them in backward with the
    RNG states captured at forward time.  With ``distribute_saved_activations``
    the first input is split 1-D across TP ranks while stored."""

    @staticmethod
    def forward(ctx, run_function, distribute_saved_activations, *args):
        ctx.run_function = run_function
        ctx.distribute = distribute_saved_activations
        ctx.fwd_cpu_rng_state = torch.get_rng_state()
        ctx.fwd_device_rng_state = _get_device_rng_state()
        ctx.fwd_tracker_states = get_cuda_rng_tracker().get_states()
        with torch.no_grad():
            outputs = run_function(*args)
        if ctx.distribute:
            ctx.input_0_shape = args[0].data.shape
            safely_set_viewless_tensor_data(
                args[0], split_tensor_into_1d_equal_chunks(args[0].data, new_buffer=True))
        ctx.save_for_backward(*[a if torch.is_tensor(a) else None for a in args])
        ctx.non_tensor_args = [None if torch.is_tensor(a) else a for a in args]
        return outputs

    @staticmethod
    def backward(ctx, *grads):
        if not torch.autograd._is_checkpoint_valid():
            raise RuntimeError("Checkpointing is not compatible with .grad(), please use .backward()")
        saved = list(ctx.saved_tensors)
        inputs = [s if s is not None else n for s, n in zip(saved, ctx.non_tensor_args)]
        if ctx.distribute:
            safely_set_viewless_tensor_data(
                inputs[0], gather_split_1d_tensor(inputs[0].data).view(ctx.input_0_shape))
        bwd_cpu = torch.get_rng_state()
        bwd_dev = _get_device_rng_state()
        bwd_tracker = get_cuda_rng_tracker().get_states()
        torch.set_rng_state(ctx.fwd_cpu_rng_state)
        _set_device_rng_state(ctx.fwd_device_rng_state)
        get_cuda_rng_tracker().set_states(ctx.fwd_tracker_states)
        detached = detach_variable(tuple(inputs))
        with torch.enable_grad():
            outputs = ctx.run_function(*detached)
        torch.set_rng_state(bwd_cpu)
        _set_device_rng_state(bwd_dev)
        get_cuda_rng_tracker().set_states(bwd_tracker)
        if isinstance(outputs, torch.Tensor):
            outputs = (outputs,)
        pairs = [(o, g) for o, g in zip(outputs, grads) if torch.is_tensor(o) and o.requires_grad]
        torch.autograd.backward([p[0] for p in pairs], [p[1] for p in pairs])
        in_grads = tuple(d.grad if isinstance(d, torch.Tensor) else None for d in detached)
        return (None, None) + in_grads


def checkpoint(function, distribute_saved_activations, *args):
    return CheckpointFunction.apply(function, distribute_saved_activations, *args)
