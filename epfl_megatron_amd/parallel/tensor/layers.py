"""Tensor-parallel layers: column/row-parallel linear and vocab-parallel embedding.

Weight shapes and attributes match the reference
(``megatron/core/tensor_parallel/layers.py:128-701``): column-parallel
weights are ``[out/tp, in]``, row-parallel ``[out, in/tp]``, row biases are
not split.

MI355X-specific design of the GEMM path (``_LinearFn``):

* Forward and dgrad GEMMs run on hipBLASLt through PyTorch, or on the
  hand-written NT GEMM (``csrc/gemm_nt.hip``) where its epilogue fuses work;
  the wgrad GEMM on the hand-written MFMA kernel (``EMA_WGRAD=hipblaslt`` for
  the library).
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
                       gather_along_first_dim,
                       gather_from_tensor_model_parallel_region,
                       reduce_from_tensor_model_parallel_region,
                       reduce_scatter_to_sequence_parallel_region,
                       scatter_to_tensor_model_parallel_region)
from .random import get_cuda_rng_tracker
from .utils import VocabUtility
from ...ops._ext import ext
from ...ops import decode_pack

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
# One 256x256 output tile per workgroup (ragged last tiles masked, so the TP=8
# FFN shards 2752 / 1376 stay on it); below one tile per CU (TP-sharded
# 7B/70B projections) the kernel splits the tokens over up to 8 workgroups per
# tile (fp32 partials + ordered reduce).  Under 32 tiles hipBLASLt is used.
_WGRAD_MIN_TILES = int(os.environ.get("EMA_WGRAD_MIN_TILES", "32"))
# Operand layouts: hipBLASLt runs "TN" problems (both operands contiguous
# along the reduction dim) 15-20 % faster than the forms PyTorch issues for
# dgrad / wgrad (profiles/r1_gemm_layouts_hipblaslt.json).  EMA_DGRAD_WT=1
# (default) keeps a K-contiguous copy of every weight, rebuilt once per
# training step by csrc/transpose.hip, so dX = dY (W^T)^T is a TN GEMM.
_DGRAD_WT = os.environ.get("EMA_DGRAD_WT", "1") != "0"
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


def _wgrad_into_main_grad(weight, grad_output_2d, input_2d, x_map=None):
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
                and (-(-N // 256)) * (-(-K // 256)) >= _WGRAD_MIN_TILES \
                and (x_map is None or x_map[0] % 32 == 0):
            ext().wgrad_gemm(grad_output_2d, input_2d, main_grad.view(N, K), accumulate,
                             list(x_map) if x_map is not None else [])
        else:
            torch.addmm(main_grad, grad_output_2d.t(), _apply_token_map(input_2d, x_map, M),
                        beta=1.0 if accumulate else 0.0, out_dtype=torch.float32, out=main_grad)
        return
    input_2d = _apply_token_map(input_2d, x_map, grad_output_2d.shape[0])
    if accumulate:
        main_grad.addmm_(grad_output_2d.t().to(main_grad.dtype), input_2d.to(main_grad.dtype))
    else:
        torch.mm(grad_output_2d.t().to(main_grad.dtype), input_2d.to(main_grad.dtype),
                 out=main_grad)


# ---- GEMM primitives ---------------------------------------------------------
# Forward / dgrad products and the fused GLU forms, with the row-group remaps
# of the SP overlap.  On the GPU they run on the hand-written NT GEMM
# (csrc/gemm_nt.hip); elsewhere (CPU / gloo tests, unsupported shapes) the
# same contract is computed with torch ops, so the chunked-overlap and fused-
# MLP control flow is exercised by the CPU equivalence tests too.
_GLU_KIND = {"swiglu": 0, "geglu": 1, "reglu": 2, "liglu": 3}


def _rows_view(t, rmap, m):
    """Logical rows [0, m) of ``t`` under a (rows, stride, offset) map, as a view."""
    if not rmap:
        return t[:m]
    R, S, O = rmap
    return t.view(-1, S, t.shape[-1])[:, O:O + R]


def _kernel_ok(a, w):
    return a.is_cuda and ext().gemm_nt_supported(a, w)


# GPU products that could not take the hand-written NT kernel (dtype / shape /
# alignment outside csrc/gemm_nt.hip's contract) and ran as torch math
# instead.  Counted per (op, reason), warned once each, reported by
# training_log; EMA_STRICT_KERNELS=1 turns them into errors.
FALLBACKS = {}
_STRICT = os.environ.get("EMA_STRICT_KERNELS", "0") == "1"


def _note_fallback(op, a, w):
    if not a.is_cuda:
        return  # CPU / gloo: torch math is the implementation
    key = (op, str(a.dtype), tuple(w.shape))
    if _STRICT:
        raise RuntimeError(f"{op}: no HIP kernel for {a.dtype} {tuple(a.shape)} x "
                           f"{tuple(w.shape)} (EMA_STRICT_KERNELS=1)")
    if key not in FALLBACKS:
        warnings.warn(f"{op}: {a.dtype} {tuple(a.shape)} x {tuple(w.shape)} is outside the "
                      "NT GEMM kernel's contract; running torch math (counted in "
                      "layers.FALLBACKS)", stacklevel=3)
    FALLBACKS[key] = FALLBACKS.get(key, 0) + 1


def fallback_report():
    """``{"op dtype shape": count}`` of GPU GEMMs that ran as torch math."""
    return {f"{k[0]} {k[1]} {list(k[2])}": v for k, v in FALLBACKS.items()}


def gemm(a, w, out=None, a_map=None, c_map=None, m=None):
    """out[c_map(q)] = a[a_map(q)] @ w^T for logical rows q < m (default: all
    rows of ``a``).  Maps: (rows, stride, offset) — see csrc/kernels.h RowMap."""
    m = m if m is not None else a.shape[0]
    if not (_NT_GEMM or a_map or c_map) and a.is_cuda and m == a.shape[0]:
        # plain product: hipBLASLt unless EMA_NT_GEMM=1 (see _NT_GEMM)
        if out is None:
            return a.matmul(w.t())
        return torch.matmul(a, w.t(), out=out)
    if _kernel_ok(a, w) and (out is None or (out.stride(1) == 1 and out.stride(0) % 8 == 0)):
        return ext().gemm_nt(a, w, out, list(a_map or []), list(c_map or []), m)
    _note_fallback("gemm", a, w)
    src = _rows_view(a, a_map, m).reshape(m, a.shape[-1])
    res = src @ w.t()
    if out is None:
        return res
    _rows_view(out, c_map, m).copy_(res.view(_rows_view(out, c_map, m).shape))
    return out


def _act(kind, x):
    return (F.silu(x), F.gelu(x), F.relu(x), x)[kind]


def gemm_glu(a, w1, kind, pre=None, y=None, c_map=None):
    """(pre, y) = (a @ w1^T, x1 * act(x2)) with x1 / x2 the up / gate halves."""
    if _kernel_ok(a, w1):
        return ext().gemm_nt_glu(a, w1, kind, pre, y, list(c_map or []))
    _note_fallback("gemm_glu", a, w1)
    p = a @ w1.t()
    f = w1.shape[0] // 2
    yy = p[:, :f] * _act(kind, p[:, f:])
    if pre is None:
        return p, yy
    _rows_view(pre, c_map, a.shape[0]).copy_(p.view(_rows_view(pre, c_map, a.shape[0]).shape))
    _rows_view(y, c_map, a.shape[0]).copy_(yy.view(_rows_view(y, c_map, a.shape[0]).shape))
    return pre, y


def gemm_dglu(g, w2t, pre, kind, out=None):
    """d(pre) = GLU backward of dAct = g @ w2t^T at the saved pre-activation
    (written into ``out`` [M, 2F] when given)."""
    if _kernel_ok(g, w2t):
        return ext().gemm_nt_dglu(g, w2t, pre, kind, out)
    _note_fallback("gemm_dglu", g, w2t)
    da = g @ w2t.t()
    f = w2t.shape[0]
    x1, x2 = pre[:, :f], pre[:, f:]
    with torch.enable_grad():
        xg = x2.detach().requires_grad_()
        a = _act(kind, xg)
        (dact,) = torch.autograd.grad(a, xg, da * x1)
    res = torch.cat([da * _act(kind, x2), dact], dim=-1)
    if out is None:
        return res
    out.copy_(res)
    return out


# ---- sequence-parallel forward overlap --------------------------------------
# Under SP a column-parallel linear all-gathers its input and a row-parallel
# linear reduce-scatters its output.  Both are split into EMA_SP_CHUNKS pieces
# of the local token rows: the all-gather of piece j+1 (resp. the reduce-
# scatter of piece j) runs on RCCL's stream while the GEMM of piece j (resp.
# j+1) runs on the compute stream; ordering is by the work handles' events.
# A gathered piece is rank-major ([tp][R] rows); the GEMM's row-group remap
# places it in natural [s, b] order (and reads the rows of one reduce-scatter
# piece out of the natural order), so no permutation copy exists.  Reference:
# megatron/core/tensor_parallel/layers.py:225-243, mappings.py:107-124 (the
# blocking forms).
_SP_CHUNKS = int(os.environ.get("EMA_SP_CHUNKS", "2"))

# Keep the forward's all-gathered SP inputs of the column-parallel products
# (QKV, fc1, the LM head) for their weight gradients instead of all-gathering
# them again in the backward (the reference re-gathers: megatron/core/
# tensor_parallel/layers.py:250-262).  That removes 2 of the 10 full-size
# [s, b, h] TP collectives per layer and micro-batch for [s, b, h] bf16 of
# HBM per product while the layer's activations live (charged by
# utils/memory_model.py).  Under full recompute the recompute forward's
# gathers are the ones kept.  --sp_regather_inputs restores the re-gather.
_SP_KEEP_GATHERED = [True]


def set_sp_keep_gathered(flag):
    _SP_KEEP_GATHERED[0] = bool(flag)


def sp_keep_gathered():
    return _SP_KEEP_GATHERED[0]


def _sp_pieces(rows_local):
    c = max(1, _SP_CHUNKS)
    return c if rows_local % c == 0 else 1


def _tp():
    world = state.get_tensor_model_parallel_world_size()
    return world, (state.get_tensor_model_parallel_group() if world > 1 else None)


def sp_allgather_gemm(x_local, w, glu_kind=None, keep=False):
    """Column-parallel forward under SP: AG(x_local) @ w^T (or the fused GLU
    pair) with the all-gather pipelined against the GEMM.  x_local [rl, K].
    ``keep``: gather into a fresh tensor and return it too (piece-major
    ``[c, tp * R, K]``; ``gathered_token_map`` pairs it with natural rows)."""
    world, group = _tp()
    rl, K = x_local.shape
    c = _sp_pieces(rl)
    R = rl // c
    dt, dev = x_local.dtype, x_local.device
    n = w.shape[0] if glu_kind is None else w.shape[0] // 2
    if glu_kind is None:
        out = torch.empty(world * rl, n, dtype=dt, device=dev)
    else:
        pre = torch.empty(world * rl, 2 * n, dtype=dt, device=dev)
        y = torch.empty(world * rl, n, dtype=dt, device=dev)
    if keep:
        g = _kept_buffer((c, world * R, K), dt, dev, group)
    else:
        g = get_global_memory_buffer().get_tensor((c, world * R, K), dt, "mpu")
    works = [comm.all_gather_into(g[j], x_local[j * R:(j + 1) * R], group=group, async_op=True)
             for j in range(c)]
    for j in range(c):
        works[j].wait()
        cmap = (R, c * R, j * R) if c > 1 else None
        if glu_kind is None:
            gemm(g[j], w, out, c_map=cmap)
        else:
            gemm_glu(g[j], w, glu_kind, pre, y, c_map=cmap)
    res = out if glu_kind is None else (pre, y)
    return (res, g) if keep else res


# EMA_LOOPBACK_KEPT_POOL=0: fresh kept-gather tensors under the loopback too (A/B)
_LOOP_KEPT_POOL = os.environ.get("EMA_LOOPBACK_KEPT_POOL", "1") != "0"


def _kept_buffer(shape, dt, dev, group):
    """Storage of an SP gather kept for the backward: a fresh tensor (the
    caching allocator recycles it after the backward), or under the
    simulated-TP loopback a pooled buffer whose simulated peers' slots are
    written once (``GlobalMemoryBuffer.get_kept``)."""
    if group is not None and _LOOP_KEPT_POOL and comm.loopback_size(group):
        return get_global_memory_buffer().get_kept(shape, dt, dev)
    return torch.empty(shape, dtype=dt, device=dev)


def gathered_token_map(rl, world):
    """Token map (``wgrad_gemm``'s x_map) from natural rows ``[rank][rl]`` of a
    sequence-parallel product to the piece-major rows ``[piece][rank][R]`` of
    ``sp_allgather_gemm``'s gather: natural q = (r, j, i) -> j * world * R +
    r * R + i.  None when the gather is in natural order (one piece)."""
    c = _sp_pieces(rl)
    if c == 1:
        return None
    R = rl // c
    return (R, c, world * R, R)


def _apply_token_map(x2, x_map, m):
    """X rows in dY's token order (the torch form of the kernel's x_map)."""
    if x_map is None:
        return x2
    R, n1, s1, s2 = x_map
    q = torch.arange(m, device=x2.device)
    grp = q // R
    idx = (grp % n1) * s1 + (grp // n1) * s2 + (q - grp * R)
    return x2.index_select(0, idx)


def sp_gemm_reducescatter(x_full, w):
    """Row-parallel forward under SP: RS(x_full @ w^T), each piece's reduce-
    scatter overlapping the next piece's GEMM.  x_full [tp * rl, K]."""
    world, group = _tp()
    M = x_full.shape[0]
    rl = M // world
    c = _sp_pieces(rl)
    R = rl // c
    n = w.shape[0]
    out = torch.empty(rl, n, dtype=x_full.dtype, device=x_full.device)
    part = torch.empty(c, world * R, n, dtype=x_full.dtype, device=x_full.device)
    works = []
    for j in range(c):
        gemm(x_full, w, part[j], a_map=(R, c * R, j * R) if c > 1 else None, m=world * R)
        works.append(comm.reduce_scatter_into(out[j * R:(j + 1) * R], part[j], group=group,
                                              async_op=True))
    for wk in works:
        wk.wait()
    return out


def _dgrad(g2, weight):
    """dX = dY W: the NT kernel on the per-step cached W^T when it applies."""
    wt = _weight_t(weight) if g2.is_cuda else None
    if wt is None:
        return g2.matmul(weight)
    return gemm(g2, wt) if _NT_GEMM else g2.matmul(wt.t())


def _fwd(x2, weight):
    return gemm(x2, weight) if (_NT_GEMM and x2.is_cuda) else x2.matmul(weight.t())


# Plain forward / dgrad GEMMs on the hand-written NT GEMM (csrc/gemm_nt.hip)
# instead of hipBLASLt: off by default — isolated, the NT kernel reaches 0.81-
# 0.90x of hipBLASLt on the 7B shapes, and the 7B step measured 28.8k tok/s
# with it vs 30.6k without (profiles/r3a_gemm_nt_bench.txt).  The fused GLU
# forms (0.98x / 1.03x of hipBLASLt + the glu kernels) stay on; the plain
# products inside the fused MLP (fc2 forward, fc1 dgrad) go to hipBLASLt
# unless a row-group remap (SP pipeline) needs the NT kernel: with them on the
# NT kernel the step measured 30.1k vs 31.0k unfused (profiles/r3c_*).
_NT_GEMM = os.environ.get("EMA_NT_GEMM", "0") == "1"


def _linear_backward(input_, weight, grad_output, use_bias, gaf, async_ar, sp, kept=None):
    """Backward of Y = X W^T (+ b) for one TP rank.  ``sp``: ``input_`` is the
    local SP shard (re-gathered here, overlapped with the dgrad GEMM) and dX is
    reduce-scattered (overlapped with the wgrad GEMM); ``async_ar``: dX is
    TP-all-reduced, overlapped with the wgrad GEMM.  ``kept``: the forward's
    gathered input (``sp_allgather_gemm(keep=True)``) with its token map; no
    re-gather (``input_`` then only gives the local shape)."""
    world, group = _tp()
    tp_group = group if world > 1 else None
    gather_handle = None
    x_map = None
    if kept is not None:
        gathered, x_map = kept
        total = gathered.view(-1, gathered.shape[-1])
    elif sp:
        shape = (input_.shape[0] * world,) + tuple(input_.shape[1:])
        total = get_global_memory_buffer().get_tensor(shape, input_.dtype, "mpu")
        gather_handle = comm.all_gather_into(total, input_, group=tp_group, async_op=True)
    else:
        total = input_
    go2 = grad_output.reshape(-1, grad_output.shape[-1])
    if not go2.is_contiguous():
        go2 = go2.contiguous()
    grad_input = _dgrad(go2, weight).view(*grad_output.shape[:-1], weight.shape[1])
    if gather_handle is not None:
        gather_handle.wait()
    ti2 = total.reshape(-1, total.shape[-1])
    handle = None
    if async_ar and tp_group is not None:
        handle = comm.all_reduce(grad_input, group=tp_group, async_op=True)
    if sp:
        if async_ar:
            raise AssertionError("sequence parallel and async all-reduce are exclusive")
        sub = torch.empty(input_.shape, dtype=grad_input.dtype, device=grad_input.device)
        handle = comm.reduce_scatter_into(sub, grad_input, group=tp_group, async_op=True)
        grad_input = sub
    grad_weight = _wgrad(weight, go2, ti2, gaf, x_map)
    grad_bias = go2.sum(dim=0) if use_bias else None
    if handle is not None:
        handle.wait()
    return grad_input, grad_weight, grad_bias


class _LinearFn(torch.autograd.Function):
    """Y = X W^T (+ b) of a column-parallel (or plain) linear; under SP the
    input all-gather is pipelined against the GEMM (``sp_allgather_gemm``)."""

    @staticmethod
    def forward(ctx, input_, weight, bias, gradient_accumulation_fusion,
                async_grad_allreduce, sequence_parallel):
        ctx.use_bias = bias is not None
        ctx.gradient_accumulation_fusion = gradient_accumulation_fusion
        ctx.async_grad_allreduce = async_grad_allreduce
        ctx.sequence_parallel = sequence_parallel
        ctx.kept_map = None
        K = input_.shape[-1]
        x2 = input_.reshape(-1, K)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        keep = sequence_parallel and sp_keep_gathered()
        ctx.keep = keep
        if sequence_parallel:
            world = state.get_tensor_model_parallel_world_size()
            out = sp_allgather_gemm(x2, weight, keep=keep)
            if keep:
                out, gathered = out
                ctx.input_shape = tuple(input_.shape)
                ctx.kept_map = gathered_token_map(x2.shape[0], world)
                ctx.save_for_backward(gathered, weight)
            lead = (input_.shape[0] * world,) + tuple(input_.shape[1:-1])
        else:
            out = _fwd(x2, weight)
            lead = tuple(input_.shape[:-1])
        if not keep:
            ctx.save_for_backward(input_, weight)
        out = out.view(*lead, weight.shape[0])
        if bias is not None:
            out = out + bias
        return out

    @staticmethod
    def backward(ctx, grad_output):
        if ctx.keep:
            gathered, weight = ctx.saved_tensors
            shape_src = torch.empty(ctx.input_shape, dtype=gathered.dtype, device="meta")
            gi, gw, gb = _linear_backward(shape_src, weight, grad_output, ctx.use_bias,
                                          ctx.gradient_accumulation_fusion,
                                          ctx.async_grad_allreduce, True,
                                          kept=(gathered, ctx.kept_map))
            return gi, gw, gb, None, None, None
        input_, weight = ctx.saved_tensors
        gi, gw, gb = _linear_backward(input_, weight, grad_output, ctx.use_bias,
                                      ctx.gradient_accumulation_fusion,
                                      ctx.async_grad_allreduce, ctx.sequence_parallel)
        return gi, gw, gb, None, None, None


class _RowParallelSPFn(torch.autograd.Function):
    """Row-parallel linear + sequence-parallel reduce-scatter in one function:
    the reduce-scatter of each output piece overlaps the next piece's GEMM
    (``sp_gemm_reducescatter``).  Backward: all-gather dY, then dgrad / wgrad."""

    @staticmethod
    def forward(ctx, input_, weight, gradient_accumulation_fusion):
        ctx.save_for_backward(input_, weight)
        ctx.gaf = gradient_accumulation_fusion
        x2 = input_.reshape(-1, input_.shape[-1])
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        world = state.get_tensor_model_parallel_world_size()
        out = sp_gemm_reducescatter(x2, weight)
        return out.view(input_.shape[0] // world, *input_.shape[1:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, grad_output):
        input_, weight = ctx.saved_tensors
        world, group = _tp()
        g_local = grad_output.reshape(-1, grad_output.shape[-1])
        if not g_local.is_contiguous():
            g_local = g_local.contiguous()
        rl, H = g_local.shape
        c = _sp_pieces(rl)
        if c == 1:
            full = gather_along_first_dim(grad_output.contiguous())
            gi, gw, _ = _linear_backward(input_, weight, full, False, ctx.gaf, False, False)
            return gi, gw, None
        # dY all-gather in c pieces, each overlapping the previous piece's dgrad
        # (the reference gathers dY in one blocking collective before any GEMM:
        # megatron/core/tensor_parallel/mappings.py:244-246).  Piece j arrives
        # rank-major; its dgrad rows go to their natural [s, b] rows by the
        # GEMM's row map, and the wgrad pairs it with X in the same piece order.
        R = rl // c
        g = get_global_memory_buffer().get_tensor((c, world * R, H), g_local.dtype, "mpu_dy")
        works = [comm.all_gather_into(g[j], g_local[j * R:(j + 1) * R], group=group,
                                      async_op=True) for j in range(c)]
        x2 = input_.reshape(-1, input_.shape[-1])
        K = x2.shape[1]
        gi = torch.empty(world * rl, K, dtype=x2.dtype, device=x2.device)
        wt = _weight_t_always(weight)
        for j in range(c):
            works[j].wait()
            gemm(g[j], wt, gi, c_map=(R, c * R, j * R))
        # dY rows are piece-major ([piece][rank][R]); X stays in natural order
        # and the wgrad reads it through a token map (no permutation copy):
        # piece-major p = (j, r, i) -> natural r * c * R + j * R + i
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        gw = _wgrad(weight, g.view(-1, H), x2, ctx.gaf, (R, world, c * R, R))
        return gi.view(*input_.shape), gw, None


# Fused GLU MLP (column-parallel fc1 -> GLU -> row-parallel fc2) on the hand-
# written NT GEMM (csrc/gemm_nt.hip): the GLU runs in the fc1 forward epilogue
# and its backward in the fc2 dgrad epilogue, so neither the activation nor its
# gradient makes an extra HBM round trip.  EMA_FUSED_MLP=0 restores the
# unfused linear + glu kernel path.
_FUSED_MLP = os.environ.get("EMA_FUSED_MLP", "1") != "0"


def fused_glu_mlp_supported(x, w1, w2, glu_kind):
    """True when ``glu_mlp`` applies (GPU: the NT kernels take every product;
    CPU: the torch forms of the same contract)."""
    if not (_FUSED_MLP and glu_kind in _GLU_KIND and w1.dtype == x.dtype
            and w2.dtype == x.dtype and w1.is_contiguous() and w2.is_contiguous()):
        return False
    H, F2 = x.shape[-1], w1.shape[0]
    Fh = F2 // 2
    if not (F2 % 2 == 0 and w1.shape[1] == H and tuple(w2.shape) == (H, Fh)):
        return False
    if not x.is_cuda:
        return True
    # fc1 forward [M,H]x[2F,H]; fc2 forward [M,F]x[H,F]; fc2 dgrad [M,H]x[F,H];
    # fc1 dgrad [M,2F]x[H,2F]: every K % 32, every N % 8, bf16 / fp16
    return (x.dtype in (torch.bfloat16, torch.float16)
            and H % 32 == 0 and Fh % 32 == 0 and H % 8 == 0 and Fh % 8 == 0)


class _GluMLPFn(torch.autograd.Function):
    """GLU(X W1^T) W2^T for one TP rank.  Without SP the result is the TP-
    partial sum (the caller reduces it, as for ``RowParallelLinear``); with SP
    the function includes both sequence-parallel collectives, each pipelined
    against its GEMM, and returns the local [s/tp] rows.

    Forward:  [SP: pipelined AG] gemm_glu (pre-act + y) -> gemm [SP: pipelined RS].
    Backward: [SP: AG dOut] gemm_dglu (fc2 dgrad, d(pre-act) through the GLU
    backward) -> fc2 wgrad -> fc1 dgrad -> [TP all-reduce or SP reduce-scatter
    of dX, async] -> fc1 wgrad.
    Reference: ``megatron/model/transformer.py:92-123`` (ParallelMLP),
    ``megatron/core/tensor_parallel/layers.py:201-317`` (the linear autograd)."""

    @staticmethod
    def forward(ctx, input_, w1, w2, kind, sequence_parallel, tp_async_allreduce, gaf):
        world = state.get_tensor_model_parallel_world_size()
        H = input_.shape[-1]
        x2 = input_.reshape(-1, H)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        kept = None
        if sequence_parallel:
            pre, y, out, kept = _sp_mlp_forward(x2, w1, w2, kind)
            lead = tuple(input_.shape[:-1])
        else:
            pre, y = gemm_glu(x2, w1, kind)
            out = gemm(y, w2)
            lead = tuple(input_.shape[:-1])
        ctx.kept = kept is not None
        ctx.input_shape = tuple(input_.shape)
        # with a kept gather the local input is not needed (shape only)
        ctx.save_for_backward(kept if kept is not None else input_, w1, w2, pre, y)
        ctx.kind, ctx.sp, ctx.tp_async, ctx.gaf = kind, sequence_parallel, tp_async_allreduce, gaf
        ctx.world = world
        return out.view(*lead, w2.shape[0])

    @staticmethod
    def backward(ctx, grad_out):
        input_, w1, w2, pre, y = ctx.saved_tensors
        world, group = _tp()
        tp_group = group if world > 1 else None
        g2 = grad_out.reshape(-1, grad_out.shape[-1])
        if not g2.is_contiguous():
            g2 = g2.contiguous()
        if ctx.sp:
            kept = None
            if ctx.kept:
                kept, input_ = input_, torch.empty(ctx.input_shape, dtype=input_.dtype,
                                                   device="meta")
            dx, gw1, gw2 = _sp_mlp_backward(input_, g2, w1, w2, pre, y, ctx.kind, ctx.gaf,
                                            kept=kept)
            return dx.view(*ctx.input_shape), gw1, gw2, None, None, None, None
        gather_handle = None
        total = input_
        # fc2 dgrad with the GLU backward in the epilogue: d(pre-act) [M, 2F]
        dpre = gemm_dglu(g2, _weight_t_always(w2), pre, ctx.kind)
        # fc1 dgrad: dX = d(pre) W1 = d(pre) (W1^T)^T
        dx = gemm(dpre, _weight_t_always(w1)).view(*total.shape[:-1], w1.shape[1])
        handle = None
        if ctx.tp_async and tp_group is not None:
            handle = comm.all_reduce(dx, group=tp_group, async_op=True)
        # weight gradients while the dX collective runs
        gw2 = _wgrad(w2, g2, y, ctx.gaf)
        if gather_handle is not None:
            gather_handle.wait()
        x2 = total.reshape(-1, total.shape[-1])
        gw1 = _wgrad(w1, dpre, x2, ctx.gaf)
        if handle is not None:
            handle.wait()
        return dx, gw1, gw2, None, None, None, None


# Sequence-parallel GLU MLP in "piece-major" row order.  The local rows are
# cut into c pieces; piece j is all-gathered on its own ([tp][R] rows, rank-
# major) and carried through fc1 + GLU -> fc2 -> reduce-scatter as it is: the
# reduce-scatter of a rank-major [tp][R] product hands every rank exactly its
# own R rows of piece j, so no GEMM needs a row remap and the token order the
# MLP sees (irrelevant to it) is (piece, rank, row).  The saved pre-activation
# and GLU output stay in that order; the backward gathers dOut and the input in
# the same pieces, so dW sums pair matching rows.  Collectives of piece j+1 run
# on RCCL's stream while piece j computes.  Reference (blocking forms):
# megatron/core/tensor_parallel/layers.py:225-243, mappings.py:107-124, 244-246.
def _sp_mlp_pieces(rl, world, n_fc1):
    """Per-rank row counts of the SP MLP pipeline's pieces: ``EMA_SP_CHUNKS``
    even pieces.  The pipeline takes any split (``EMA_SP_MLP_PIECES=r0,r1,...``
    forces one; the equivalence tests run uneven pieces).  An uneven split
    sized to the fc1 + GLU tile rounds (Llama-2-7B TP8: 736 + 1312 rows per
    rank, 1 + 2 rounds instead of 2 + 2) cut that product's piece cost from
    1.239x to 1.033x of the monolithic GEMM and the MLP forward by 8.5 %, but
    the uneven fc1 dgrad / fc2 pieces lost more: the TP8 proxy step ran 4 %
    slower (profiles/r4ab_sp_pieces.txt, profiles/r4ac_sp_pieces_proxy_ab.txt),
    so the split stays even."""
    forced = os.environ.get("EMA_SP_MLP_PIECES")
    if forced:
        sizes = [int(v) for v in forced.split(",")]
        if sum(sizes) == rl and all(v > 0 for v in sizes):
            return sizes
    c = _sp_pieces(rl)
    return [rl // c] * c


def _sp_mlp_forward(x_local, w1, w2, kind):
    world, group = _tp()
    rl, H = x_local.shape
    dt, dev = x_local.dtype, x_local.device
    F = w2.shape[1]
    sizes = _sp_mlp_pieces(rl, world, 2 * F)
    offs = [sum(sizes[:j]) for j in range(len(sizes))]
    # piece-major buffers: piece j's gathered rows at [world * off_j, world * (off_j + R_j));
    # kept for the fc1 wgrad (same piece order as every other MLP tensor)
    if sp_keep_gathered():
        g = _kept_buffer((world * rl, H), dt, dev, group)
    else:
        g = get_global_memory_buffer().get_tensor((world * rl, H), dt, "mpu")
    gp = [g[world * o:world * (o + r)] for o, r in zip(offs, sizes)]
    works = [comm.all_gather_into(gp[j], x_local[o:o + r], group=group, async_op=True)
             for j, (o, r) in enumerate(zip(offs, sizes))]
    pre = torch.empty(world * rl, 2 * F, dtype=dt, device=dev)
    y = torch.empty(world * rl, F, dtype=dt, device=dev)
    part = torch.empty(world * rl, w2.shape[0], dtype=dt, device=dev)
    out = torch.empty(rl, w2.shape[0], dtype=dt, device=dev)
    rs = []
    for j, (o, r) in enumerate(zip(offs, sizes)):
        rows = slice(world * o, world * (o + r))
        works[j].wait()
        gemm_glu(gp[j], w1, kind, pre[rows], y[rows])
        gemm(y[rows], w2, part[rows])
        rs.append(comm.reduce_scatter_into(out[o:o + r], part[rows], group=group,
                                           async_op=True))
    for w in rs:
        w.wait()
    return pre, y, out, (g if sp_keep_gathered() else None)


def _sp_mlp_backward(input_, g_local, w1, w2, pre, y, kind, gaf, kept=None):
    """Backward of ``_sp_mlp_forward``: dOut and X gathered in the forward's
    pieces; per piece the fc2 dgrad (+ GLU backward) and the fc1 dgrad run while
    the next piece's gathers fly, and dX's reduce-scatter of piece j overlaps
    piece j+1; both wgrads run last over all pieces."""
    world, group = _tp()
    x_local = input_.reshape(-1, input_.shape[-1])
    if kept is None and not x_local.is_contiguous():
        x_local = x_local.contiguous()
    rl, H = x_local.shape
    dt, dev = g_local.dtype, g_local.device
    F = w2.shape[1]
    sizes = _sp_mlp_pieces(rl, world, 2 * F)
    offs = [sum(sizes[:j]) for j in range(len(sizes))]
    pieces = list(zip(offs, sizes))
    buf = get_global_memory_buffer()
    g2 = buf.get_tensor((world * rl, g_local.shape[1]), g_local.dtype, "mpu_dy")
    gw = [comm.all_gather_into(g2[world * o:world * (o + r)], g_local[o:o + r], group=group,
                               async_op=True) for o, r in pieces]
    if kept is not None:  # the forward's gather (piece-major, as the re-gather would be)
        xt, xw = kept, []
    else:
        xt = buf.get_tensor((world * rl, H), dt, "mpu")
        xw = [comm.all_gather_into(xt[world * o:world * (o + r)], x_local[o:o + r], group=group,
                                   async_op=True) for o, r in pieces]
    dpre = torch.empty(world * rl, 2 * F, dtype=dt, device=dev)
    dxp = torch.empty(world * rl, H, dtype=dt, device=dev)
    dx = torch.empty(rl, H, dtype=dt, device=dev)
    w2t, w1t = _weight_t_always(w2), _weight_t_always(w1)
    rs = []
    for j, (o, r) in enumerate(pieces):
        rows = slice(world * o, world * (o + r))
        gw[j].wait()
        gemm_dglu(g2[rows], w2t, pre[rows], kind, dpre[rows])
        gemm(dpre[rows], w1t, dxp[rows])
        rs.append(comm.reduce_scatter_into(dx[o:o + r], dxp[rows], group=group, async_op=True))
    gw2 = _wgrad(w2, g2, y, gaf)
    for w in xw:
        w.wait()
    gw1 = _wgrad(w1, dpre, xt, gaf)
    for w in rs:
        w.wait()
    return dx, gw1, gw2


def _weight_t_always(weight):
    """W^T, cached per training step when possible, else built now."""
    wt = _weight_t(weight) if weight.is_cuda else None
    if wt is not None:
        return wt
    return _transpose(weight) if _tn_ok(weight) else weight.t().contiguous()


def _wgrad(weight, g2, x2, gaf, x_map=None):
    """Weight gradient of Y = X W^T: into main_grad (returns None) or as a
    tensor.  ``x_map``: X's rows are a token permutation of dY's
    (``wgrad_gemm``'s x_map, e.g. ``gathered_token_map``)."""
    if gaf and hasattr(weight, "main_grad"):
        _wgrad_into_main_grad(weight, g2, x2, x_map)
        _notify_grad_ready(weight)
        return None
    return g2.t().matmul(_apply_token_map(x2, x_map, g2.shape[0]))


def glu_mlp(input_, w1, w2, glu_kind, *, sequence_parallel, tp_async_allreduce,
            gradient_accumulation_fusion):
    """Per-rank GLU MLP through the fused kernels (see ``_GluMLPFn``).  Without
    SP the caller reduces the returned partial output across the TP group."""
    return _GluMLPFn.apply(input_, w1, w2, _GLU_KIND[glu_kind], sequence_parallel,
                           tp_async_allreduce, gradient_accumulation_fusion)


# Decode-sized inference batches (<= 32 token rows, no autograd): the weight-
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
    if m > 32 or not weight.is_contiguous() or not ext().skinny_gemm_supported(m, n, k):
        return None
    # K = 4096 / 8192 run the persistent skinny kernel, faster than hipBLASLt up
    # to the LM head at 16 rows; the per-block form loses to hipBLASLt's wide
    # tiles on wide outputs (profiles/r3i_skinny_persistent_ab.txt)
    if k not in (4096, 8192) and ((m > 8 and n > 16384) or (m > 4 and n > 24576)):
        return None
    x2 = input_.reshape(m, k)
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    wp = decode_pack.packed(weight)  # decode-packed copy (ops/decode_pack.py) or None
    out = ext().skinny_gemm(x2, weight if wp is None else wp, wp is not None)
    out = out.view(*input_.shape[:-1], weight.shape[0])
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
        if self.sequence_parallel_enabled:
            # GEMM + reduce-scatter pipelined in pieces (_RowParallelSPFn)
            output_ = _RowParallelSPFn.apply(input_parallel, self.weight,
                                             self.gradient_accumulation_fusion)
        else:
            output_parallel = _skinny_linear(input_parallel, self.weight, None, False)
            if output_parallel is None:
                output_parallel = _LinearFn.apply(input_parallel, self.weight, None,
                                                  self.gradient_accumulation_fusion, False, False)
            output_ = reduce_from_tensor_model_parallel_region(output_parallel)
        if not self.skip_bias_add:
            output = output_ + self.bias if self.bias is not None else output_
            output_bias = None
        else:
            output = output_
            output_bias = self.bias
        return output, output_bias
