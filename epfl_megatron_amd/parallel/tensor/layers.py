"""Tensor-parallel layers: column/row-parallel linear and vocab-parallel embedding.

Weight shapes and attributes match the reference
(``megatron/core/tensor_parallel/layers.py:128-701``): column-parallel
weights are ``[out/tp, in]``, row-parallel ``[out, in/tp]``, row biases are
not split.

MI355X-specific design of the GEMM path (``_LinearFn``):

* Forward and dgrad GEMMs run on hipBLASLt through PyTorch (``EMA_GEMM=tuned``
  switches to ``ops/gemm.py``'s per-shape solution timing); the wgrad GEMM
  on the hand-written MFMA kernel (``EMA_WGRAD=hipblaslt`` for the library).
* With ``gradient_accumulation_fusion`` the weight gradient is a
  bf16 x bf16 -> fp32 GEMM written **in place** into the fp32 ``main_grad``
  view of the DDP bucket —
  no separate wgrad tensor, no accumulate kernel, and no zero-fill (the first
  micro-batch stores with beta = 0; reference N8 / apex
  ``fused_weight_gradient_mlp_cuda``).  Immediately after
  enqueueing it we signal the DDP bucket manager, which can start that
  bucket's RCCL reduction while backward continues (the reference only
  reduces after the whole backward).
* Under sequence parallelism the input all-gather for the wgrad is issued
  before the dgrad GEMM and the dgrad reduce-scatter is overlapped with the
  wgrad GEMM, using async RCCL work handles (RCCL runs on its own HIP stream;
  ordering comes from events, not from ``CUDA_DEVICE_MAX_CONNECTIONS``).
"""
import math
import os
import warnings

import torch
import torch.nn.functional as F
from torch.nn.parameter import Parameter

from .. import state, comm
from ..buffers import divide, get_global_memory_buffer
from .mappings import (copy_to_tensor_model_parallel_region,
                       gather_from_tensor_model_parallel_region,
                       reduce_from_tensor_model_parallel_region,
                       reduce_scatter_to_sequence_parallel_region,
                       scatter_to_tensor_model_parallel_region)
from .random import get_cuda_rng_tracker
from .utils import VocabUtility
from ...ops._ext import ext
from ...ops import gemm as tuned_gemm

_MODEL_PARALLEL_ATTRIBUTE_DEFAULTS = {
    "tensor_model_parallel": False,
    "partition_dim": -1,
    "partition_stride": 1,
}


def param_is_not_tensor_parallel_duplicate(param):
    return (getattr(param, "tensor_model_parallel", False)
            or state.get_tensor_model_parallel_rank() == 0)


def set_tensor_model_parallel_attributes(tensor, is_parallel, dim, stride):
    for attr in _MODEL_PARALLEL_ATTRIBUTE_DEFAULTS:
        if hasattr(tensor, attr):
            raise AssertionError(f"tensor already has attribute {attr}")
    tensor.tensor_model_parallel = is_parallel
    tensor.partition_dim = dim
    tensor.partition_stride = stride


def set_defaults_if_not_set_tensor_model_parallel_attributes(tensor):
    for attr, val in _MODEL_PARALLEL_ATTRIBUTE_DEFAULTS.items():
        if not hasattr(tensor, attr):
            setattr(tensor, attr, val)


def copy_tensor_model_parallel_attributes(dst, src):
    for attr in _MODEL_PARALLEL_ATTRIBUTE_DEFAULTS:
        if hasattr(src, attr):
            setattr(dst, attr, getattr(src, attr))


def _initialize_affine_weight_gpu(weight, init_method, partition_dim, stride=1):
    set_tensor_model_parallel_attributes(weight, True, partition_dim, stride)
    with get_cuda_rng_tracker().fork():
        init_method(weight)


def _initialize_affine_weight_cpu(weight, output_size, input_size, per_partition_size,
                                  partition_dim, init_method, stride=1,
                                  return_master_weight=False, params_dtype=torch.float32):
    """Initialise the full master weight on CPU, then keep this rank's slice —
    results are independent of the TP degree (used by --use_cpu_initialization)."""
    set_tensor_model_parallel_attributes(weight, True, partition_dim, stride)
    master = torch.empty(output_size, input_size, dtype=torch.float, requires_grad=False)
    init_method(master)
    master = master.to(dtype=params_dtype)
    per_stride = divide(per_partition_size, stride)
    pieces = torch.split(master, per_stride, dim=partition_dim)
    rank = state.get_tensor_model_parallel_rank()
    world = state.get_tensor_model_parallel_world_size()
    mine = pieces[rank::world]
    with torch.no_grad():
        torch.cat(mine, dim=partition_dim, out=weight)
    return master if return_master_weight else None


def _default_device():
    return torch.cuda.current_device() if torch.cuda.is_available() else "cpu"


class VocabParallelEmbedding(torch.nn.Module):
    """Embedding sharded along the vocab dim; out-of-shard ids contribute zeros
    and the partial rows are summed with one TP all-reduce."""

    def __init__(self, num_embeddings, embedding_dim, *, init_method=torch.nn.init.xavier_normal_,
                 params_dtype=torch.float32, use_cpu_initialization=False,
                 perform_initialization=True):
        super().__init__()
        self.num_embeddings = num_embeddings
        self.embedding_dim = embedding_dim
        self.tensor_model_parallel_size = state.get_tensor_model_parallel_world_size()
        self.vocab_start_index, self.vocab_end_index = \
            VocabUtility.vocab_range_from_global_vocab_size(
                num_embeddings, state.get_tensor_model_parallel_rank(),
                self.tensor_model_parallel_size)
        self.num_embeddings_per_partition = self.vocab_end_index - self.vocab_start_index
        if use_cpu_initialization or not torch.cuda.is_available():
            self.weight = Parameter(torch.empty(self.num_embeddings_per_partition, embedding_dim,
                                                dtype=params_dtype))
            if perform_initialization:
                _initialize_affine_weight_cpu(self.weight, num_embeddings, embedding_dim,
                                              self.num_embeddings_per_partition, 0, init_method,
                                              params_dtype=params_dtype)
            else:
                set_tensor_model_parallel_attributes(self.weight, True, 0, 1)
        else:
            self.weight = Parameter(torch.empty(self.num_embeddings_per_partition, embedding_dim,
                                                device=_default_device(), dtype=params_dtype))
            if perform_initialization:
                _initialize_affine_weight_gpu(self.weight, init_method, partition_dim=0)
            else:
                set_tensor_model_parallel_attributes(self.weight, True, 0, 1)

    def forward(self, input_):
        if self.tensor_model_parallel_size > 1:
            mask = (input_ < self.vocab_start_index) | (input_ >= self.vocab_end_index)
            ids = input_.clone() - self.vocab_start_index
            ids[mask] = 0
        else:
            ids = input_
        out = F.embedding(ids, self.weight)
        if self.tensor_model_parallel_size > 1:
            out = out.masked_fill(mask.unsqueeze(-1), 0.0)
        return reduce_from_tensor_model_parallel_region(out)


def _notify_grad_ready(param):
    cb = getattr(param, "_main_grad_ready", None)
    if cb is not None:
        cb()


# Weight-gradient GEMM backend: the hand-written MFMA kernel (csrc/gemm_wgrad.hip,
# default; EMA_WGRAD=hipblaslt for the library): 1.11-1.40 PF isolated vs
# 0.94-1.16 PF and 28.3k vs 26.7k tokens/s in the 7B step (profiles/r2_wgrad_ab.txt).
_WGRAD_KERNEL = os.environ.get("EMA_WGRAD", "hip").lower() == "hip"
# One 256x256 output tile per workgroup; below one tile per CU (TP-sharded
# 7B/70B projections) the kernel splits the tokens over up to 8 workgroups per
# tile (fp32 partials + ordered reduce).  Under 32 tiles hipBLASLt is used.
_WGRAD_MIN_TILES = int(os.environ.get("EMA_WGRAD_MIN_TILES", "32"))
# EMA_GEMM=tuned routes all three products through ops/gemm.py (per-shape
# solution timing).  Off by default: in the full 7B step it measured 22.4k vs
# 22.9k tokens/s for PyTorch's own hipBLASLt calls (profiles/r1_gemm_ab.txt) —
# isolated timings with hot caches do not predict in-model kernel times.
_TUNED_GEMM = os.environ.get("EMA_GEMM", "torch").lower() == "tuned"
# Operand layouts: hipBLASLt runs "TN" problems (both operands contiguous
# along the reduction dim) 15-20 % faster than the forms PyTorch issues for
# dgrad / wgrad (profiles/r1_gemm_layouts_hipblaslt.json).  EMA_DGRAD_WT=1
# (default) keeps a K-contiguous copy of every weight, rebuilt once per
# training step by csrc/transpose.hip, so dX = dY (W^T)^T is a TN GEMM.
# EMA_WGRAD_TN=1 also transposes dY and X so that
# main_grad (+)= (dY^T) (X^T)^T is one.
_DGRAD_WT = os.environ.get("EMA_DGRAD_WT", "1") != "0"
_WGRAD_TN = os.environ.get("EMA_WGRAD_TN", "0") == "1"
_WEIGHT_T_GEN = [0]  # 0: no training step in flight -> no cached transposes


def new_weight_transpose_generation():
    """Called by ``train_step``: parameters may have changed since the last step,
    so every cached W^T is rebuilt on its first use in this step."""
    _WEIGHT_T_GEN[0] += 1


def _tn_ok(t):
    return (t.is_cuda and t.dim() == 2 and t.dtype in (torch.bfloat16, torch.float16)
            and t.is_contiguous() and t.data_ptr() % 16 == 0
            and ext().transpose16_supported(t.shape[0], t.shape[1]))


def _transpose(t):
    out = torch.empty(t.shape[1], t.shape[0], dtype=t.dtype, device=t.device)
    ext().transpose16(t, out)
    return out


def _weight_t(weight):
    """Contiguous W^T built at most once per training step (None: not applicable)."""
    gen = _WEIGHT_T_GEN[0]
    if not (_DGRAD_WT and gen > 0 and _tn_ok(weight)):
        return None
    key = (gen, weight.data_ptr(), weight._version)
    cached = getattr(weight, "_wt_cache", None)
    if cached is not None and cached[0] == key:
        return cached[1]
    shape = (weight.shape[1], weight.shape[0])
    if cached is not None and tuple(cached[1].shape) == shape and cached[1].dtype == weight.dtype:
        wt = cached[1]
    else:
        wt = torch.empty(shape, dtype=weight.dtype, device=weight.device)
    ext().transpose16(weight, wt)
    weight._wt_cache = (key, wt)
    return wt


def _wgrad_into_main_grad(weight, grad_output_2d, input_2d):
    """main_grad[out, in] (+)= dY^T @ X with fp32 accumulation, in place.

    ``weight._mg_fresh`` (set by ``DistributedDataParallel.zero_grad_buffer``
    instead of zero-filling the buffer) makes the first contribution of a step
    a plain store (beta = 0): no fill kernel, no read of the old values.  On
    the GPU the hand-written MFMA kernel (``csrc/gemm_wgrad.hip``) is used for
    every shape it tiles (split over tokens when it has fewer tiles than CUs);
    others go to hipBLASLt through ``torch.addmm``.
    """
    main_grad = weight.main_grad
    accumulate = not getattr(weight, "_mg_fresh", False)
    weight._mg_fresh = False
    if main_grad.is_cuda and grad_output_2d.dtype in (torch.bfloat16, torch.float16):
        M, N = grad_output_2d.shape
        K = input_2d.shape[1]
        if _WGRAD_KERNEL and main_grad.is_contiguous() and grad_output_2d.is_contiguous() \
                and input_2d.is_contiguous() and ext().wgrad_supported(M, N, K) \
                and (N // 256) * (K // 256) >= _WGRAD_MIN_TILES:
            ext().wgrad_gemm(grad_output_2d, input_2d, main_grad.view(N, K), accumulate)
        elif _TUNED_GEMM:
            tuned_gemm.wgrad(main_grad.view(N, K), grad_output_2d, input_2d, accumulate)
        elif _WGRAD_TN and _tn_ok(grad_output_2d) and _tn_ok(input_2d):
            # token-contiguous operands: dY^T [N, M] and X^T [K, M] -> TN GEMM
            torch.addmm(main_grad, _transpose(grad_output_2d), _transpose(input_2d).t(),
                        beta=1.0 if accumulate else 0.0, out_dtype=torch.float32,
                        out=main_grad)
        else:
            torch.addmm(main_grad, grad_output_2d.t(), input_2d, beta=1.0 if accumulate else 0.0,
                        out_dtype=torch.float32, out=main_grad)
    elif accumulate:
        main_grad.addmm_(grad_output_2d.t().to(main_grad.dtype), input_2d.to(main_grad.dtype))
    else:
        torch.mm(grad_output_2d.t().to(main_grad.dtype), input_2d.to(main_grad.dtype),
                 out=main_grad)


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input_, weight, bias, gradient_accumulation_fusion,
                async_grad_allreduce, sequence_parallel):
        ctx.save_for_backward(input_, weight)
        ctx.use_bias = bias is not None
        ctx.gradient_accumulation_fusion = gradient_accumulation_fusion
        ctx.async_grad_allreduce = async_grad_allreduce
        ctx.sequence_parallel = sequence_parallel
        if sequence_parallel:
            world = state.get_tensor_model_parallel_world_size()
            shape = (input_.shape[0] * world,) + tuple(input_.shape[1:])
            total = get_global_memory_buffer().get_tensor(shape, input_.dtype, "mpu")
            comm.all_gather_into(total, input_, group=state.get_tensor_model_parallel_group())
        else:
            total = input_
        if total.is_cuda and _TUNED_GEMM:
            x2 = total.reshape(-1, total.shape[-1])
            out = tuned_gemm.linear_fwd(x2, weight).view(*total.shape[:-1], weight.shape[0])
        else:
            out = torch.matmul(total, weight.t())
        if bias is not None:
            out = out + bias
        return out

    @staticmethod
    def backward(ctx, grad_output):
        input_, weight = ctx.saved_tensors
        tp_group = state.get_tensor_model_parallel_group() \
            if state.get_tensor_model_parallel_world_size() > 1 else None
        gather_handle = None
        if ctx.sequence_parallel:
            world = state.get_tensor_model_parallel_world_size()
            shape = (input_.shape[0] * world,) + tuple(input_.shape[1:])
            total = get_global_memory_buffer().get_tensor(shape, input_.dtype, "mpu")
            gather_handle = comm.all_gather_into(total, input_, group=tp_group, async_op=True)
        else:
            total = input_
        if grad_output.is_cuda and _TUNED_GEMM:
            g2 = grad_output.reshape(-1, grad_output.shape[-1])
            grad_input = tuned_gemm.linear_dgrad(g2, weight).view(
                *grad_output.shape[:-1], weight.shape[1])
        else:
            wt = _weight_t(weight) if grad_output.is_cuda else None
            grad_input = grad_output.matmul(weight) if wt is None else grad_output.matmul(wt.t())
        if gather_handle is not None:
            gather_handle.wait()
        go2 = grad_output.reshape(-1, grad_output.shape[-1])
        ti2 = total.reshape(-1, total.shape[-1])
        handle = None
        if ctx.async_grad_allreduce and tp_group is not None:
            handle = comm.all_reduce(grad_input, group=tp_group, async_op=True)
        sub_grad_input = None
        if ctx.sequence_parallel:
            if ctx.async_grad_allreduce:
                raise AssertionError("sequence parallel and async all-reduce are exclusive")
            world = state.get_tensor_model_parallel_world_size()
            sub_grad_input = torch.empty((input_.shape[0],) + tuple(input_.shape[1:]),
                                         dtype=input_.dtype, device=input_.device)
            handle = comm.reduce_scatter_into(sub_grad_input, grad_input, group=tp_group,
                                              async_op=True)
        if ctx.gradient_accumulation_fusion and hasattr(weight, "main_grad"):
            _wgrad_into_main_grad(weight, go2, ti2)
            grad_weight = None
            _notify_grad_ready(weight)
        else:
            grad_weight = go2.t().matmul(ti2)
        grad_bias = go2.sum(dim=0) if ctx.use_bias else None
        if ctx.sequence_parallel:
            if handle is not None:
                handle.wait()
            return sub_grad_input, grad_weight, grad_bias, None, None, None
        if handle is not None:
            handle.wait()
        return grad_input, grad_weight, grad_bias, None, None, None


# Decode-sized inference batches (<= 16 token rows, no autograd): the weight-
# streaming HIP GEMM (csrc/skinny_gemm.hip) instead of hipBLASLt's skinny
# tiles (profiles/r2c_skinny_gemm.txt).  EMA_SKINNY_GEMM=0 disables it.
_SKINNY = os.environ.get("EMA_SKINNY_GEMM", "1") != "0"


def _skinny_linear(input_, weight, bias, sequence_parallel):
    """Y = X W^T (+ bias) through the skinny kernel when it applies, else None."""
    if not (_SKINNY and input_.is_cuda and not sequence_parallel and not torch.is_grad_enabled()
            and input_.dtype in (torch.bfloat16, torch.float16) and weight.dtype == input_.dtype):
        return None
    k = input_.shape[-1]
    m = input_.numel() // k
    n = weight.shape[0]
    if m > 16 or not weight.is_contiguous() or not ext().skinny_gemm_supported(m, n, k):
        return None
    if (m > 8 and n > 16384) or (m > 4 and n > 24576):  # hipBLASLt's wide tiles win there
        return None
    x2 = input_.reshape(m, k)
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    out = ext().skinny_gemm(x2, weight).view(*input_.shape[:-1], weight.shape[0])
    return out if bias is None else out + bias


def linear_with_grad_accumulation_and_async_allreduce(input, weight, bias,
                                                      gradient_accumulation_fusion,
                                                      async_grad_allreduce,
                                                      sequence_parallel_enabled):
    out = _skinny_linear(input, weight, bias, sequence_parallel_enabled)
    if out is not None:
        return out
    return _LinearFn.apply(input, weight, bias, gradient_accumulation_fusion,
                           async_grad_allreduce, sequence_parallel_enabled)


def _make_weight(rows, cols, dtype, use_cpu_init):
    if use_cpu_init or not torch.cuda.is_available():
        return Parameter(torch.empty(rows, cols, dtype=dtype))
    return Parameter(torch.empty(rows, cols, device=_default_device(), dtype=dtype))


def _make_bias(n, dtype, use_cpu_init):
    if use_cpu_init or not torch.cuda.is_available():
        b = Parameter(torch.empty(n, dtype=dtype))
    else:
        b = Parameter(torch.empty(n, device=_default_device(), dtype=dtype))
    with torch.no_grad():
        b.zero_()
    return b


class ColumnParallelLinear(torch.nn.Module):
    """Y = XA + b with A split along its output dim: A = [A_1 ... A_p]."""

    def __init__(self, input_size, output_size, *, bias=True, gather_output=True,
                 init_method=torch.nn.init.xavier_normal_, stride=1, keep_master_weight_for_test=False,
                 skip_bias_add=False, async_tensor_model_parallel_allreduce=True,
                 params_dtype=torch.float32, use_cpu_initialization=False,
                 perform_initialization=True, gradient_accumulation_fusion=False,
                 sequence_parallel_enabled=False):
        super().__init__()
        self.input_size = input_size
        self.output_size = output_size
        self.gather_output = gather_output
        world = state.get_tensor_model_parallel_world_size()
        self.output_size_per_partition = divide(output_size, world)
        self.skip_bias_add = skip_bias_add
        self.weight = _make_weight(self.output_size_per_partition, input_size, params_dtype,
                                   use_cpu_initialization)
        if perform_initialization:
            if use_cpu_initialization or not torch.cuda.is_available():
                self.master_weight = _initialize_affine_weight_cpu(
                    self.weight, output_size, input_size, self.output_size_per_partition, 0,
                    init_method, stride=stride, return_master_weight=keep_master_weight_for_test,
                    params_dtype=params_dtype)
            else:
                _initialize_affine_weight_gpu(self.weight, init_method, partition_dim=0,
                                              stride=stride)
        else:
            set_tensor_model_parallel_attributes(self.weight, True, 0, stride)
        if bias:
            self.bias = _make_bias(self.output_size_per_partition, params_dtype,
                                   use_cpu_initialization)
            set_tensor_model_parallel_attributes(self.bias, True, 0, stride)
        else:
            self.register_parameter("bias", None)
        self.async_tensor_model_parallel_allreduce = (
            async_tensor_model_parallel_allreduce and world > 1)
        if sequence_parallel_enabled and world <= 1:
            warnings.warn("`sequence_parallel_enabled` is set to `True`, but tensor model "
                          "parallel size is 1; disabling it.")
            sequence_parallel_enabled = False
        self.sequence_parallel_enabled = sequence_parallel_enabled
        self.gradient_accumulation_fusion = gradient_accumulation_fusion
        if self.async_tensor_model_parallel_allreduce and self.sequence_parallel_enabled:
            raise RuntimeError("`async_tensor_model_parallel_allreduce` and "
                               "`sequence_parallel_enabled` cannot be enabled at the same time.")

    def forward(self, input_):
        bias = self.bias if not self.skip_bias_add else None
        if self.async_tensor_model_parallel_allreduce or self.sequence_parallel_enabled:
            input_parallel = input_
        else:
            input_parallel = copy_to_tensor_model_parallel_region(input_)
        output_parallel = _skinny_linear(input_parallel, self.weight, bias,
                                         self.sequence_parallel_enabled)
        if output_parallel is None:
            output_parallel = _LinearFn.apply(input_parallel, self.weight, bias,
                                              self.gradient_accumulation_fusion,
                                              self.async_tensor_model_parallel_allreduce,
                                              self.sequence_parallel_enabled)
        if self.gather_output:
            if self.sequence_parallel_enabled:
                raise AssertionError("gather_output is incompatible with sequence parallelism")
            output = gather_from_tensor_model_parallel_region(output_parallel)
        else:
            output = output_parallel
        output_bias = self.bias if self.skip_bias_add else None
        return output, output_bias


class RowParallelLinear(torch.nn.Module):
    """Y = XA + b with A split along its input dim; partial outputs are summed
    with an all-reduce (or reduce-scattered along the sequence under SP)."""

    def __init__(self, input_size, output_size, *, bias=True, input_is_parallel=False,
                 init_method=torch.nn.init.xavier_normal_, stride=1,
                 keep_master_weight_for_test=False, skip_bias_add=False,
                 params_dtype=torch.float32, use_cpu_initialization=False,
                 perform_initialization=True, gradient_accumulation_fusion=False,
                 sequence_parallel_enabled=False):
        super().__init__()
        self.input_size = input_size
        self.output_size = output_size
        self.input_is_parallel = input_is_parallel
        world = state.get_tensor_model_parallel_world_size()
        self.input_size_per_partition = divide(input_size, world)
        self.skip_bias_add = skip_bias_add
        self.gradient_accumulation_fusion = gradient_accumulation_fusion
        self.sequence_parallel_enabled = sequence_parallel_enabled
        if self.sequence_parallel_enabled and not self.input_is_parallel:
            raise RuntimeError("To enable `sequence_parallel_enabled`, `input_is_parallel` "
                               "must be `True`")
        self.weight = _make_weight(output_size, self.input_size_per_partition, params_dtype,
                                   use_cpu_initialization)
        if perform_initialization:
            if use_cpu_initialization or not torch.cuda.is_available():
                self.master_weight = _initialize_affine_weight_cpu(
                    self.weight, output_size, input_size, self.input_size_per_partition, 1,
                    init_method, stride=stride, return_master_weight=keep_master_weight_for_test,
                    params_dtype=params_dtype)
            else:
                _initialize_affine_weight_gpu(self.weight, init_method, partition_dim=1,
                                              stride=stride)
        else:
            set_tensor_model_parallel_attributes(self.weight, True, 1, stride)
        if bias:
            self.bias = _make_bias(output_size, params_dtype, use_cpu_initialization)
            setattr(self.bias, "sequence_parallel", sequence_parallel_enabled)
        else:
            self.register_parameter("bias", None)

    def forward(self, input_):
        if self.input_is_parallel:
            input_parallel = input_
        else:
            if self.sequence_parallel_enabled:
                raise AssertionError("sequence parallelism needs a parallel input")
            input_parallel = scatter_to_tensor_model_parallel_region(input_)
        output_parallel = _skinny_linear(input_parallel, self.weight, None, False)
        if output_parallel is None:
            output_parallel = _LinearFn.apply(input_parallel, self.weight, None,
                                              self.gradient_accumulation_fusion, False, False)
        if self.sequence_parallel_enabled:
            output_ = reduce_scatter_to_sequence_parallel_region(output_parallel)
        else:
            output_ = reduce_from_tensor_model_parallel_region(output_parallel)
        if not self.skip_bias_add:
            output = output_ + self.bias if self.bias is not None else output_
            output_bias = None
        else:
            output = output_
            output_bias = self.bias
        return output, output_bias
