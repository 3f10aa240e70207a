"""Transformer stack: attention, MLP, layer, and the per-stage layer container.

Module tree and parameter names match the reference
(``megatron/model/transformer.py:77-1251``) so checkpoints interchange:
``layers.{i}.input_layernorm``, ``self_attention.query_key_value``,
``self_attention.dense``, ``post_attention_layernorm``,
``mlp.dense_h_to_4h``, ``mlp.dense_4h_to_h``, ``[mlp_layernorm]``,
``[output_layernorm]``, ``final_layernorm``.

MI355X hot path (flash attention on): RMSNorm/LayerNorm HIP kernel ->
QKV GEMM (hipBLASLt) -> k-only RoPE pass + FlashAttention-2 HIP kernel (Q RoPE fused) reading
the fused ``[s, b, ng, r+2, hd]`` QKV tensor through strides (native GQA, no
K/V expansion, no rearrange copies) -> dense GEMM -> residual -> norm ->
fc1 GEMM -> fused GLU/GeLU HIP kernel -> fc2 GEMM -> residual.

Fixes relative to the reference: KV cache stores *rotated* keys (D1), K/V
are cached at KV-head count (D2), full recompute forwards ``position_ids``
(D5), the RoPE table lives on the device (D10), GLU never routes through the
bias-GeLU fusion (D15).
"""
import math
import os
from contextlib import nullcontext

import torch
import torch.nn.functional as F

from .. import global_vars
from ..parallel import state
from ..parallel.buffers import divide, make_viewless_tensor
from ..parallel import tensor as tp
from ..ops.dropout import bias_dropout_add
from ..utils.trace import trace_range, tracing
from ..ops.norms import RMSNorm, MixedFusedLayerNorm, _param_sync, rms_norm
from ..ops.rope import rope_table, apply_rope_ref, rope_qkv_inplace, rope_qkv
from ..ops._ext import use_native, ext
from ..parallel.context import chunk_position_ids, ring_attention
from ..ops.attention import flash_attn_qkvpacked, flash_attn_func, flash_decode_cached
from ..ops.activations import glu, bias_gelu, gelu
from ..ops import decode_pack
from ..ops.softmax import FusedScaleMaskSoftmax
from .enums import AttnMaskType, AttnType, LayerType, ModelType, PositionEmbeddingType
from .module import MegatronModule
from .utils import attention_mask_func, erf_gelu


# Decode steps (one new token per sequence, <= 32 sequences, any TP) run each
# layer as 5 weight-streaming launches with the elementwise work fused in
# (csrc/skinny_gemm.hip): [RMSNorm + QKV + RoPE + KV-cache write] ->
# decode attention -> [dense + residual] -> [RMSNorm + fc1 + GLU] ->
# [fc2 + residual].  EMA_DECODE_FUSED=0 keeps the unfused kernels.
_DECODE_FUSED = os.environ.get("EMA_DECODE_FUSED", "1") != "0"


def _linear_kwargs(args):
    return dict(params_dtype=args.params_dtype,
                use_cpu_initialization=bool(args.use_cpu_initialization),
                perform_initialization=args.perform_initialization,
                gradient_accumulation_fusion=args.gradient_accumulation_fusion,
                sequence_parallel_enabled=args.sequence_parallel)


def _make_norm(args, dim=None):
    dim = dim or args.hidden_size
    if args.use_rms_norm:
        return RMSNorm(dim, eps=args.layernorm_epsilon, sequence_parallel=args.sequence_parallel)
    return MixedFusedLayerNorm(dim, eps=args.layernorm_epsilon,
                               no_persist_layer_norm=args.no_persist_layer_norm,
                               sequence_parallel=args.sequence_parallel)


class DropPath(MegatronModule):
    """Per-sample stochastic depth on ``[s, b, h]``."""

    def __init__(self, drop_prob=0.0):
        super().__init__()
        self.drop_prob = drop_prob

    def forward(self, x):
        if self.drop_prob == 0.0 or not self.training:
            return x
        keep = 1 - self.drop_prob
        shape = (1, x.shape[1]) + (1,) * (x.ndim - 2)
        mask = (keep + torch.rand(shape, dtype=x.dtype, device=x.device)).floor_()
        return x.div(keep) * mask


class ParallelMLP(MegatronModule):
    def __init__(self, init_method, output_layer_init_method, args, world_size=None):
        super().__init__()
        self.glu_activation = args.glu_activation
        self.use_bias = args.use_bias
        self.bias_gelu_fusion = args.bias_gelu_fusion
        self.onnx_safe = bool(args.onnx_safe)
        width = 2 * args.ffn_hidden_size if args.glu_activation else args.ffn_hidden_size
        self.dense_h_to_4h = tp.ColumnParallelLinear(
            args.hidden_size, width, bias=args.use_bias, gather_output=False,
            init_method=init_method, skip_bias_add=True,
            async_tensor_model_parallel_allreduce=args.async_tensor_model_parallel_allreduce,
            **_linear_kwargs(args))
        self.dense_4h_to_h = tp.RowParallelLinear(
            args.ffn_hidden_size, args.hidden_size, bias=args.use_bias, input_is_parallel=True,
            init_method=output_layer_init_method, skip_bias_add=True, **_linear_kwargs(args))

    def _fused_ok(self, x):
        fc1, fc2 = self.dense_h_to_4h, self.dense_4h_to_h
        if not self.glu_activation or self.use_bias:
            return False
        if not torch.is_grad_enabled() and x.numel() // x.shape[-1] < 256:
            # decode rows: the weight-streaming skinny GEMM (<= 32 rows) or
            # hipBLASLt's narrow tiles; the NT kernel's 256-row tiles would run
            # mostly empty (batch-32 decode 5.7k -> 4.5k tok/s with them)
            return False
        return tp.fused_glu_mlp_supported(x, fc1.weight, fc2.weight, self.glu_activation)

    def forward(self, hidden_states):
        if self._fused_ok(hidden_states):
            # fc1 + GLU + fc2 on the NT GEMM with the GLU in its epilogues
            fc1, fc2 = self.dense_h_to_4h, self.dense_4h_to_h
            _param_sync(fc1.weight, fc2.weight)  # module pre-hooks are bypassed
            x = hidden_states
            if not (fc1.async_tensor_model_parallel_allreduce or fc1.sequence_parallel_enabled):
                x = tp.copy_to_tensor_model_parallel_region(x)
            out = tp.glu_mlp(x, fc1.weight, fc2.weight, self.glu_activation,
                             sequence_parallel=fc1.sequence_parallel_enabled,
                             tp_async_allreduce=fc1.async_tensor_model_parallel_allreduce,
                             gradient_accumulation_fusion=fc1.gradient_accumulation_fusion)
            if not fc2.sequence_parallel_enabled:  # (SP: reduce-scattered inside)
                out = tp.reduce_from_tensor_model_parallel_region(out)
            return out, None
        inter, bias = self.dense_h_to_4h(hidden_states)
        if self.glu_activation:
            if bias is not None:
                inter = inter + bias
            inter = glu(inter, self.glu_activation)
        elif self.bias_gelu_fusion:
            inter = bias_gelu(bias, inter)
        else:
            if bias is not None:
                inter = inter + bias
            inter = erf_gelu(inter) if self.onnx_safe else gelu(inter)
        return self.dense_4h_to_h(inter)


class CoreAttention(MegatronModule):
    """Non-flash attention: QK^T (baddbmm) -> fused scale/mask/softmax HIP
    kernel -> dropout -> PV.  Keeps the reference's query-key layer scaling."""

    def __init__(self, layer_number, attn_mask_type=AttnMaskType.padding, args=None,
                 world_size=None):
        super().__init__()
        self.fp16, self.bf16 = args.fp16, args.bf16
        self.apply_query_key_layer_scaling = args.apply_query_key_layer_scaling
        self.attention_softmax_in_fp32 = args.attention_softmax_in_fp32 or \
            self.apply_query_key_layer_scaling
        self.layer_number = max(1, layer_number)
        self.attn_mask_type = attn_mask_type
        self.sequence_parallel = args.sequence_parallel
        world_size = world_size or state.get_tensor_model_parallel_world_size()
        projection_size = args.kv_channels * args.num_attention_heads
        self.hidden_size_per_partition = divide(projection_size, world_size)
        self.hidden_size_per_attention_head = divide(projection_size, args.num_attention_heads)
        self.num_attention_heads_per_partition = divide(args.num_attention_heads, world_size)
        coeff = None
        self.norm_factor = math.sqrt(self.hidden_size_per_attention_head)
        if self.apply_query_key_layer_scaling:
            coeff = self.layer_number
            self.norm_factor *= coeff
        self.scale_mask_softmax = FusedScaleMaskSoftmax(
            self.fp16, self.bf16, self.attn_mask_type, args.masked_softmax_fusion,
            attention_mask_func, self.attention_softmax_in_fp32, coeff)
        self.attention_dropout = torch.nn.Dropout(args.attention_dropout)

    def forward(self, query_layer, key_layer, value_layer, attention_mask):
        # q: [sq, b, np, hn], k/v: [sk, b, np, hn]
        sq, b, np_, hn = query_layer.shape
        sk = key_layer.shape[0]
        q = query_layer.reshape(sq, b * np_, hn).transpose(0, 1)
        k = key_layer.reshape(sk, b * np_, hn).transpose(0, 1)
        scores = torch.empty(b * np_, sq, sk, dtype=q.dtype, device=q.device)
        scores = torch.baddbmm(scores, q, k.transpose(1, 2), beta=0.0,
                               alpha=1.0 / self.norm_factor).view(b, np_, sq, sk)
        if self.attn_mask_type == AttnMaskType.causal and sq != sk:
            # Inference with a KV cache: explicit bottom-right aligned mask.
            i = torch.arange(sq, device=q.device)[:, None]
            j = torch.arange(sk, device=q.device)[None, :]
            attention_mask = (j > i + (sk - sq))[None, None]
            probs = self.scale_mask_softmax.forward_torch_softmax(scores, attention_mask)
        else:
            probs = self.scale_mask_softmax(scores, attention_mask)
        if not self.sequence_parallel:
            with tp.get_cuda_rng_tracker().fork():
                probs = self.attention_dropout(probs)
        else:
            probs = self.attention_dropout(probs)
        v = value_layer.reshape(sk, b * np_, hn).transpose(0, 1)
        ctx = torch.bmm(probs.view(b * np_, sq, sk).to(v.dtype), v)
        ctx = ctx.view(b, np_, sq, hn).permute(2, 0, 1, 3).contiguous()
        return ctx.view(sq, b, self.hidden_size_per_partition)


class ParallelAttention(MegatronModule):
    """Self (or cross) attention with fused, GQA-grouped QKV projection."""

    def __init__(self, init_method, output_layer_init_method, layer_number,
                 attention_type=AttnType.self_attn, attn_mask_type=AttnMaskType.padding,
                 world_size=None, args=None):
        super().__init__()
        world_size = world_size or state.get_tensor_model_parallel_world_size()
        self.layer_number = max(1, layer_number)
        self.attention_type = attention_type
        self.attn_mask_type = attn_mask_type
        self.params_dtype = args.params_dtype
        self.sequence_parallel = args.sequence_parallel
        self.use_flash_attn = args.use_flash_attn
        self.num_attention_heads = args.num_attention_heads
        self.num_attention_heads_kv = args.num_attention_heads_kv
        self.seq_length = args.seq_length
        if self.use_flash_attn:
            if attention_type != AttnType.self_attn:
                raise AssertionError("FlashAttention code path only supports self-attention")
            if attn_mask_type != AttnMaskType.causal:
                raise AssertionError("FlashAttention code path only supports causal mask")
        hd = args.kv_channels
        projection_size = hd * args.num_attention_heads
        self.hidden_size_per_attention_head = divide(projection_size, args.num_attention_heads)
        self.num_attention_heads_per_partition = divide(args.num_attention_heads, world_size)
        self.num_groups_per_partition = divide(args.num_attention_heads_kv, world_size)
        self.q_per_group = args.num_attention_heads // args.num_attention_heads_kv
        if attention_type == AttnType.self_attn:
            qkv_size = hd * args.num_attention_heads + 2 * hd * args.num_attention_heads_kv
            self.query_key_value = tp.ColumnParallelLinear(
                args.hidden_size, qkv_size, bias=args.use_bias, gather_output=False,
                init_method=init_method,
                async_tensor_model_parallel_allreduce=args.async_tensor_model_parallel_allreduce,
                **_linear_kwargs(args))
        else:
            self.query = tp.ColumnParallelLinear(
                args.hidden_size, projection_size, bias=args.use_bias, gather_output=False,
                init_method=init_method,
                async_tensor_model_parallel_allreduce=args.async_tensor_model_parallel_allreduce,
                **_linear_kwargs(args))
            self.key_value = tp.ColumnParallelLinear(
                args.hidden_size, 2 * projection_size, bias=args.use_bias, gather_output=False,
                init_method=init_method,
                async_tensor_model_parallel_allreduce=args.async_tensor_model_parallel_allreduce,
                **_linear_kwargs(args))
        self.core_attention = CoreAttention(self.layer_number, attn_mask_type, args, world_size)
        self.checkpoint_core_attention = args.recompute_granularity == "selective"
        self.dense = tp.RowParallelLinear(
            projection_size, args.hidden_size, bias=args.use_bias, input_is_parallel=True,
            init_method=output_layer_init_method, skip_bias_add=True, **_linear_kwargs(args))
        self.position_embedding_type = args.position_embedding_type
        self.rope_len = max(args.seq_length, args.max_position_embeddings or 0)
        self.rope_scaling = args.rope_scaling_factor
        # context parallelism: this rank holds one contiguous sequence chunk
        self.cp_group = state.get_context_parallel_group() \
            if attention_type == AttnType.self_attn else None

    # -- helpers ---------------------------------------------------------
    def _rope(self, device):
        if self.position_embedding_type != PositionEmbeddingType.rotary:
            return None
        return rope_table(self.hidden_size_per_attention_head, self.rope_len, device,
                          scaling_factor=self.rope_scaling)

    def _split_qkv(self, mixed):
        sq, b = mixed.shape[:2]
        hd, g, r = self.hidden_size_per_attention_head, self.num_groups_per_partition, \
            self.q_per_group
        qkv = mixed.view(sq, b, g, r + 2, hd)
        q = qkv[:, :, :, :r, :].reshape(sq, b, g * r, hd)
        k = qkv[:, :, :, r, :]
        v = qkv[:, :, :, r + 1, :]
        return q, k, v

    def _expand_kv(self, t):
        return t.repeat_interleave(self.q_per_group, dim=2) if self.q_per_group > 1 else t

    def _allocate_kv(self, max_len, max_batch, device):
        shape = (max_len, max_batch, self.num_groups_per_partition,
                 self.hidden_size_per_attention_head)
        return (torch.empty(shape, dtype=self.params_dtype, device=device),
                torch.empty(shape, dtype=self.params_dtype, device=device))

    def _core(self, q, k, v, attention_mask):
        if self.checkpoint_core_attention and self.training:
            return tp.checkpoint(lambda *a: self.core_attention(*a), False, q, k, v,
                                 attention_mask)
        return self.core_attention(q, k, v, attention_mask)

    # -- forward ---------------------------------------------------------
    def forward(self, hidden_states, attention_mask, encoder_output=None, inference_params=None,
                position_ids=None):
        if self.attention_type != AttnType.self_attn:
            return self._cross_forward(hidden_states, attention_mask, encoder_output)
        mixed, _ = self.query_key_value(hidden_states)
        rope = self._rope(mixed.device)
        if inference_params is not None:
            ctx = self._inference_forward(mixed, attention_mask, inference_params, position_ids,
                                          rope)
        elif self.cp_group is not None:
            ctx = self._context_parallel_forward(mixed, position_ids, rope, attention_mask)
        elif self.use_flash_attn:
            rng = tp.get_cuda_rng_tracker().fork() if not self.sequence_parallel else nullcontext()
            with rng:
                # packed documents (--reset_attention_mask): the mask arrives as
                # int32 [2, b, s] document bounds (utils/misc.py doc_bounds)
                docs = attention_mask if (attention_mask is not None and
                                          attention_mask.dtype == torch.int32) else None
                ctx = flash_attn_qkvpacked(mixed, self.num_groups_per_partition, self.q_per_group,
                                           self.hidden_size_per_attention_head, causal=True,
                                           rope=rope, position_ids=position_ids, doc_bounds=docs)
        else:
            q, k, v = self._split_qkv(mixed)
            if rope is not None:
                q = apply_rope_ref(q, rope[0], rope[1], position_ids)
                k = apply_rope_ref(k, rope[0], rope[1], position_ids)
            ctx = self._core(q, self._expand_kv(k), self._expand_kv(v), attention_mask)
        return self.dense(ctx)

    def _context_parallel_forward(self, mixed, position_ids, rope, attention_mask=None):
        """Causal self-attention of this rank's zig-zag share of the sequence
        over the whole sequence: RoPE at the share's global positions, then the
        K/V ring (``parallel/context.py``) with the FlashAttention pair kernels.
        ``attention_mask``: None, or (``--reset_attention_mask``) the WHOLE
        sequence's int32 [2, b, S] document bounds."""
        sq, b = mixed.shape[:2]
        if rope is not None:
            if position_ids is None:
                position_ids = chunk_position_ids(sq, b, mixed.device)
            g, r, hd = self.num_groups_per_partition, self.q_per_group, \
                self.hidden_size_per_attention_head
            mixed = rope_qkv(mixed.view(sq, b, g, r + 2, hd), rope[0], rope[1],
                             position_ids.long()).view(sq, b, -1)
        q, k, v = self._split_qkv(mixed)
        docs = attention_mask if (attention_mask is not None and
                                  attention_mask.dtype == torch.int32) else None
        o = ring_attention(q.transpose(0, 1), k.transpose(0, 1), v.transpose(0, 1),
                           self.cp_group, causal=True, zigzag=True, docs=docs)
        return o.transpose(0, 1).reshape(sq, b, -1)

    def _inference_forward(self, mixed, attention_mask, ip, position_ids, rope):
        s0 = ip.sequence_len_offset
        b0 = ip.batch_size_offset
        if rope is not None and use_native(mixed) and mixed.is_contiguous() and \
                not (torch.is_grad_enabled() and mixed.requires_grad):
            # one in-place HIP pass over q and k of the fused projection, with
            # the true positions, BEFORE caching (fixes D1)
            sq_, b_ = mixed.shape[:2]
            rope_qkv_inplace(mixed.view(sq_, b_, self.num_groups_per_partition,
                                        self.q_per_group + 2, self.hidden_size_per_attention_head),
                             rope[0], rope[1], position_ids, offset=s0)
            rope = None
        q, k, v = self._split_qkv(mixed)
        sq, b = q.shape[:2]
        if self.layer_number not in ip.key_value_memory_dict:
            ip.key_value_memory_dict[self.layer_number] = self._allocate_kv(
                ip.max_sequence_len, ip.max_batch_size, mixed.device)
        kmem, vmem = ip.key_value_memory_dict[self.layer_number]
        if rope is not None:
            # Rotate with the true positions BEFORE caching (fixes D1).
            q = apply_rope_ref(q, rope[0], rope[1], position_ids, offset=s0)
            k = apply_rope_ref(k, rope[0], rope[1], position_ids, offset=s0)
        if getattr(ip, "device_offset", None) is not None and sq == 1:
            # hipGraph decode step (inference/hip_graph.py): cache slot and key
            # count live in device tensors, so no launch depends on the step
            # (on the CPU the static-buffer step runs eagerly: reference attention)
            if q.is_cuda and not (use_native(q) and q.shape[-1] in (64, 128)):
                raise NotImplementedError("hipGraph decode needs the native decode attention "
                                          "kernel (GPU, bf16/fp16, head_dim 64 or 128)")
            kc, vc = kmem[:, b0:b0 + b], vmem[:, b0:b0 + b]
            kc.index_copy_(0, ip.device_offset, k)
            vc.index_copy_(0, ip.device_offset, v)
            o = flash_decode_cached(q.transpose(0, 1), kc.transpose(0, 1), vc.transpose(0, 1),
                                    ip.device_kv_len)
            return o.transpose(0, 1).reshape(sq, b, -1)
        kmem[s0:s0 + sq, b0:b0 + b] = k
        vmem[s0:s0 + sq, b0:b0 + b] = v
        keys = kmem[:s0 + sq, b0:b0 + b]
        vals = vmem[:s0 + sq, b0:b0 + b]
        if self.use_flash_attn:
            o = flash_attn_func(q.transpose(0, 1), keys.transpose(0, 1), vals.transpose(0, 1),
                                causal=True)
            return o.transpose(0, 1).reshape(sq, b, -1)
        return self.core_attention(q, self._expand_kv(keys), self._expand_kv(vals),
                                   attention_mask)

    def _cross_forward(self, hidden_states, attention_mask, encoder_output):
        kv, _ = self.key_value(encoder_output)
        sk, b = kv.shape[:2]
        kv = kv.view(sk, b, self.num_attention_heads_per_partition,
                     2 * self.hidden_size_per_attention_head)
        k, v = tp.split_tensor_along_last_dim(kv, 2)
        q, _ = self.query(hidden_states)
        q = q.view(q.shape[0], q.shape[1], self.num_attention_heads_per_partition,
                   self.hidden_size_per_attention_head)
        ctx = self._core(q, k, v, attention_mask)
        return self.dense(ctx)


class ParallelTransformerLayer(MegatronModule):
    """One transformer block (pre-LN by default; post-LN, Falcon parallel
    attention/MLP and parallel layernorm supported)."""

    def __init__(self, init_method, output_layer_init_method, layer_number,
                 layer_type=LayerType.encoder, self_attn_mask_type=AttnMaskType.padding,
                 drop_path_rate=0.0, world_size=None, hidden_dropout=0.0, args=None):
        super().__init__()
        self.layer_number = layer_number
        self.layer_type = layer_type
        self.apply_residual_connection_post_layernorm = \
            args.apply_residual_connection_post_layernorm
        self.fp32_residual_connection = args.fp32_residual_connection
        self.parallel_layernorm = args.parallel_layernorm
        self.parallel_attn = args.parallel_attn
        self.use_post_ln = args.use_post_ln
        self.use_bias = args.use_bias
        self.params_dtype = args.params_dtype
        self.input_layernorm = torch.nn.Identity() if args.use_post_ln else _make_norm(args)
        self.output_layernorm = _make_norm(args) if args.use_post_ln else torch.nn.Identity()
        if self.parallel_layernorm:
            self.mlp_layernorm = _make_norm(args)
        self.self_attention = ParallelAttention(
            init_method, output_layer_init_method, layer_number, attention_type=AttnType.self_attn,
            attn_mask_type=self_attn_mask_type, world_size=world_size, args=args)
        self.hidden_dropout = hidden_dropout
        self.drop_path = DropPath(drop_path_rate) if drop_path_rate > 0.0 else None
        if not args.parallel_attn:
            self.post_attention_layernorm = _make_norm(args)
        if layer_type == LayerType.decoder:
            self.inter_attention = ParallelAttention(
                init_method, output_layer_init_method, layer_number,
                attention_type=AttnType.cross_attn, world_size=world_size, args=args)
            self.post_inter_attention_layernorm = _make_norm(args)
        self.mlp = ParallelMLP(init_method, output_layer_init_method, args, world_size)

    def _add(self, x, bias, residual, make_viewless=False, x2=None):
        """residual + dropout(x [+ x2] [+ bias]): one fused HIP pass on the GPU
        (``ops.dropout``, Philox-consistent with the TP RNG tracker); ``x2`` is
        the Falcon parallel block's attention output."""
        if self.drop_path is None:
            out = bias_dropout_add(x, bias, residual, self.hidden_dropout, self.training, x2=x2)
        else:
            if x2 is not None:
                x = x + x2
            if bias is not None:
                x = x + bias
            p = self.hidden_dropout if self.training else 0.0
            if p > 0.0:
                x = F.dropout(x, p=p, training=True)
            out = residual + self.drop_path(x)
        if make_viewless:
            out = make_viewless_tensor(out, requires_grad=out.requires_grad, keep_graph=True)
        return out

    def _fused_residual_ok(self):
        """Plain pre-LN block with nothing between the residual add and the
        next norm (no dropout / drop-path / post-LN variants) -> the adds fold
        into the norm kernels (``ops.norms.norm_residual``)."""
        return (not self.use_post_ln and not self.parallel_attn and not self.parallel_layernorm
                and not self.apply_residual_connection_post_layernorm
                and not self.fp32_residual_connection and self.layer_type == LayerType.encoder
                and (self.hidden_dropout == 0.0 or not self.training) and self.drop_path is None
                and hasattr(self.input_layernorm, "forward_residual"))

    def _decode_fused_ok(self, hidden_states, ip):
        """One decode step of a plain pre-RMSNorm rotary GLU block (any TP size,
        no sequence parallelism: a decode step has one row per sequence)."""
        if not (_DECODE_FUSED and ip is not None and not torch.is_grad_enabled()
                and hidden_states.is_cuda and hidden_states.dim() == 3
                and hidden_states.shape[0] == 1 and hidden_states.shape[1] <= 32
                and hidden_states.dtype in (torch.bfloat16, torch.float16)
                and self._fused_residual_ok()):
            return False
        sa, mlp = self.self_attention, self.mlp
        if not (isinstance(self.input_layernorm, RMSNorm)
                and isinstance(self.post_attention_layernorm, RMSNorm)
                and sa.attention_type == AttnType.self_attn
                and sa.position_embedding_type == PositionEmbeddingType.rotary
                and sa.query_key_value.bias is None and sa.dense.bias is None
                and mlp.glu_activation and not mlp.use_bias
                and not sa.dense.sequence_parallel_enabled
                and not mlp.dense_4h_to_h.sequence_parallel_enabled
                and sa.hidden_size_per_attention_head in (64, 128)):
            return False
        C = ext()
        b, H = hidden_states.shape[1], hidden_states.shape[2]
        wq, wo = sa.query_key_value.weight, sa.dense.weight
        w1, w2 = mlp.dense_h_to_4h.weight, mlp.dense_4h_to_h.weight
        ws = (wq, wo, w1, w2, self.input_layernorm.weight, self.post_attention_layernorm.weight)
        if any(w.dtype != hidden_states.dtype or not w.is_contiguous() for w in ws):
            return False
        F2 = w1.shape[0]
        return (F2 % 16 == 0 and C.skinny_gemm_supported(b, wq.shape[0], H)
                and C.skinny_gemm_supported(b, H, wo.shape[1])
                and C.skinny_gemm_supported(b, F2, H) and C.skinny_gemm_supported(b, H, F2 // 2))

    def _forward_decode_fused(self, hidden_states, ip, position_ids):
        sa, mlp = self.self_attention, self.mlp
        ln1, ln2 = self.input_layernorm, self.post_attention_layernorm
        C = ext()
        _, b, H = hidden_states.shape
        x = hidden_states.reshape(b, H)
        if not x.is_contiguous():
            x = x.contiguous()
        if sa.layer_number not in ip.key_value_memory_dict:
            ip.key_value_memory_dict[sa.layer_number] = sa._allocate_kv(
                ip.max_sequence_len, ip.max_batch_size, x.device)
        kmem, vmem = ip.key_value_memory_dict[sa.layer_number]
        b0, s0 = ip.batch_size_offset, ip.sequence_len_offset
        kc, vc = kmem[:, b0:b0 + b], vmem[:, b0:b0 + b]
        cos, sin = sa._rope(x.device)
        if position_ids is None:
            pos = torch.full((b, 1), s0, dtype=torch.long, device=x.device)
        else:
            pos = position_ids[:, -1:].long()
        graph = getattr(ip, "device_offset", None) is not None
        ng, r, hd = sa.num_groups_per_partition, sa.q_per_group, sa.hidden_size_per_attention_head
        # weights in the decode-packed layout when the shape allows (ops/decode_pack.py)
        wq, wo = sa.query_key_value.weight, sa.dense.weight
        w1, w2 = mlp.dense_h_to_4h.weight, mlp.dense_4h_to_h.weight
        # 17-32 rows: the norm runs as its own kernel and the projections take
        # the un-normed two-row-block forms (the normed ones spill their 2 x 16
        # X fragments: profiles/r4ai_skinny_mb.txt)
        sep = b > 16
        pq, po = decode_pack.packed(wq), decode_pack.packed(wo)
        # the half-unit tail of the form that will run (normed for <= 16 rows)
        tail = C.skinny_glu_half_tail(w1.shape[0] // 2, w1.shape[1], not sep, b)
        p1, p2 = decode_pack.packed(w1, glu=True, half_tail=tail), decode_pack.packed(w2)
        xq = rms_norm(x, ln1.weight, ln1.eps) if sep else x
        q = C.skinny_qkv_rope_cache(xq, wq if pq is None else pq, None if sep else ln1.weight,
                                    ln1.eps, ng, r, hd,
                                    cos, sin, pos, kc, vc,
                                    ip.device_offset if graph else None, 0 if graph else s0,
                                    pq is not None)
        q4 = q.view(b, 1, ng * r, hd)
        if graph:
            o = flash_decode_cached(q4, kc.transpose(0, 1), vc.transpose(0, 1), ip.device_kv_len)
        else:
            o = flash_attn_func(q4, kc[:s0 + 1].transpose(0, 1), vc[:s0 + 1].transpose(0, 1),
                                causal=True)
        # Row-parallel dense / fc2 under TP: each rank's product is a partial
        # sum; TP rank 0 alone adds the residual in its epilogue, so one
        # all-reduce of [b, H] yields partial sums + residual (reference
        # RowParallelLinear + bias-dropout-add: megatron/model/transformer.py:
        # 707-730, megatron/core/tensor_parallel/layers.py:665-701).
        # (one persistent launch with grid barriers for these three products was
        # measured 2.6x slower than the three launches: profiles/r3x_decode_mlp_fused.txt)
        first = state.get_tensor_model_parallel_rank() == 0
        h2 = C.skinny_norm_gemm(o.reshape(b, -1), wo if po is None else po, None, 0.0,
                                x if first else None, po is not None)
        h2 = tp.reduce_from_tensor_model_parallel_region(h2)
        y = C.skinny_norm_glu(rms_norm(h2, ln2.weight, ln2.eps) if sep else h2,
                              w1 if p1 is None else p1, None if sep else ln2.weight, ln2.eps,
                              tp.layers._GLU_KIND[mlp.glu_activation], p1 is not None, tail)
        h3 = C.skinny_norm_gemm(y, w2 if p2 is None else p2, None, 0.0, h2 if first else None,
                                p2 is not None)
        h3 = tp.reduce_from_tensor_model_parallel_region(h3)
        return h3.view(1, b, H)

    def _forward_fused_residual(self, hidden_states, attention_mask, inference_params,
                                position_ids):
        ln_out, residual = self.input_layernorm.forward_residual(hidden_states)
        attn_out, attn_bias = self.self_attention(ln_out, attention_mask,
                                                  inference_params=inference_params,
                                                  position_ids=position_ids)
        if attn_bias is None:
            ln_out, ln_in = self.post_attention_layernorm.forward_residual(attn_out, residual)
        else:
            ln_in = self._add(attn_out, attn_bias, residual)
            ln_out = self.post_attention_layernorm(ln_in)
        mlp_out, mlp_bias = self.mlp(ln_out)
        return self._add(mlp_out, mlp_bias, ln_in, make_viewless=True)

    def forward(self, hidden_states, attention_mask, encoder_output=None, enc_dec_attn_mask=None,
                inference_params=None, position_ids=None):
        if tracing():
            with trace_range(f"layer{self.layer_number}"):
                return self._forward(hidden_states, attention_mask, encoder_output,
                                     enc_dec_attn_mask, inference_params, position_ids)
        return self._forward(hidden_states, attention_mask, encoder_output, enc_dec_attn_mask,
                             inference_params, position_ids)

    def _forward(self, hidden_states, attention_mask, encoder_output=None, enc_dec_attn_mask=None,
                 inference_params=None, position_ids=None):
        if self._decode_fused_ok(hidden_states, inference_params):
            return self._forward_decode_fused(hidden_states, inference_params, position_ids)
        if self._fused_residual_ok():
            return self._forward_fused_residual(hidden_states, attention_mask, inference_params,
                                                position_ids)
        ln_out = self.input_layernorm(hidden_states)
        if self.fp32_residual_connection and ln_out.dtype == torch.float32:
            ln_out = ln_out.to(self.params_dtype)
        attn_out, attn_bias = self.self_attention(ln_out, attention_mask,
                                                  inference_params=inference_params,
                                                  position_ids=position_ids)
        residual = ln_out if self.apply_residual_connection_post_layernorm else hidden_states
        if self.parallel_layernorm:
            ln_out = self.mlp_layernorm(hidden_states)
        if self.parallel_attn:
            ln_in = attn_out
        else:
            ln_in = self._add(attn_out, attn_bias, residual)
            ln_out = self.post_attention_layernorm(ln_in)
        if self.layer_type == LayerType.decoder:
            attn_out, attn_bias = self.inter_attention(ln_out, enc_dec_attn_mask,
                                                       encoder_output=encoder_output)
            residual = ln_out if self.apply_residual_connection_post_layernorm else ln_in
            ln_in = self._add(attn_out, attn_bias, residual)
            ln_out = self.post_inter_attention_layernorm(ln_in)
        mlp_out, mlp_bias = self.mlp(ln_out)
        if self.parallel_attn:  # Falcon: residual + dropout(mlp + attn) in one pass
            out = self._add(mlp_out, mlp_bias, residual, make_viewless=True, x2=attn_out)
            return self.output_layernorm(out)
        elif self.apply_residual_connection_post_layernorm:
            residual = ln_out
        else:
            residual = ln_in
        out = self._add(mlp_out, mlp_bias, residual, make_viewless=True)
        return self.output_layernorm(out)


class NoopTransformerLayer(MegatronModule):
    """Stands in for a stage with zero layers (standalone embedding stage)."""

    def __init__(self, layer_number):
        super().__init__()
        self.layer_number = layer_number

    def forward(self, hidden_states, attention_mask, encoder_output=None, enc_dec_attn_mask=None,
                inference_params=None, position_ids=None):
        return hidden_states.clone()


def _get_num_layers(args, is_encoder_and_decoder_model, is_decoder=False):
    if state.get_pipeline_model_parallel_world_size() > 1:
        first_stage_empty = args.standalone_embedding_stage and \
            state.get_pipeline_model_parallel_rank() == 0
        if is_encoder_and_decoder_model:
            if args.pipeline_model_parallel_split_rank is None:
                raise AssertionError("split rank required for encoder-decoder pipelines")
            enc_ranks = args.pipeline_model_parallel_split_rank - \
                (1 if args.standalone_embedding_stage else 0)
            dec_ranks = args.transformer_pipeline_model_parallel_size - enc_ranks
            if args.encoder_num_layers % enc_ranks or args.decoder_num_layers % dec_ranks:
                raise AssertionError("encoder/decoder layers must divide their ranks")
            if state.is_pipeline_stage_before_split():
                return 0 if first_stage_empty else args.encoder_num_layers // enc_ranks
            return args.decoder_num_layers // dec_ranks
        if args.num_layers % args.transformer_pipeline_model_parallel_size != 0:
            raise AssertionError("num_layers must be divisible by "
                                 "transformer_pipeline_model_parallel_size")
        return 0 if first_stage_empty else \
            args.num_layers // args.transformer_pipeline_model_parallel_size
    return args.decoder_num_layers if is_decoder else args.encoder_num_layers


class ParallelTransformer(MegatronModule):
    """The layers owned by this pipeline stage (+ final norm on the last stage)."""

    def __init__(self, init_method, output_layer_init_method, layer_type=LayerType.encoder,
                 self_attn_mask_type=AttnMaskType.padding, pre_process=True, post_process=True,
                 drop_path_rate=0.0, args=None, model_type=None):
        super().__init__()
        world_size = state.get_tensor_model_parallel_world_size()
        self.layer_type = layer_type
        self.model_type = model_type
        self.pre_process = pre_process
        self.post_process = post_process
        self.input_tensor = None
        self.recompute_granularity = args.recompute_granularity
        self.recompute_method = args.recompute_method
        self.recompute_num_layers = args.recompute_num_layers
        self.distribute_saved_activations = args.distribute_saved_activations and \
            not args.sequence_parallel
        self.sequence_parallel = args.sequence_parallel
        self.use_post_ln = args.use_post_ln
        self.num_layers = _get_num_layers(args, model_type == ModelType.encoder_and_decoder,
                                          layer_type == LayerType.decoder)
        drop_path_rates = torch.linspace(0, drop_path_rate, args.num_layers).tolist()
        if args.lima_dropout:
            dropouts = torch.linspace(0, args.hidden_dropout, args.num_layers).tolist()
        else:
            dropouts = [args.hidden_dropout] * args.num_layers

        if args.virtual_pipeline_model_parallel_size is not None:
            if args.num_layers % args.virtual_pipeline_model_parallel_size != 0:
                raise AssertionError("num_layers_per_stage must be divisible by "
                                     "virtual_pipeline_model_parallel_size")
            self.num_layers //= args.virtual_pipeline_model_parallel_size
            offset = state.get_virtual_pipeline_model_parallel_rank() * \
                (args.num_layers // args.virtual_pipeline_model_parallel_size) + \
                state.get_pipeline_model_parallel_rank() * self.num_layers
        elif model_type == ModelType.encoder_and_decoder and \
                state.get_pipeline_model_parallel_world_size() > 1:
            prank = state.get_pipeline_model_parallel_rank()
            if layer_type == LayerType.encoder:
                offset = prank * self.num_layers
            else:
                offset = (prank - args.pipeline_model_parallel_split_rank) * self.num_layers
        else:
            offset = state.get_pipeline_model_parallel_rank() * self.num_layers

        if self.num_layers == 0:
            self.num_layers = 1
            self.layers = torch.nn.ModuleList([NoopTransformerLayer(1)])
        else:
            self.layers = torch.nn.ModuleList([
                ParallelTransformerLayer(
                    init_method, output_layer_init_method, i + 1 + offset, layer_type=layer_type,
                    self_attn_mask_type=self_attn_mask_type,
                    drop_path_rate=drop_path_rates[i + offset] if i + offset < len(drop_path_rates)
                    else 0.0,
                    world_size=world_size,
                    hidden_dropout=dropouts[min(i + offset, len(dropouts) - 1)], args=args)
                for i in range(self.num_layers)])
        if self.post_process:
            self.final_layernorm = _make_norm(args)

    def _get_layer(self, n):
        return self.layers[n]

    def set_input_tensor(self, input_tensor):
        self.input_tensor = input_tensor

    def _run(self, start, end):
        def fwd(hidden, mask, enc_out, enc_dec_mask, position_ids):
            for i in range(start, end):
                hidden = self.layers[i](hidden, mask, encoder_output=enc_out,
                                        enc_dec_attn_mask=enc_dec_mask,
                                        position_ids=position_ids)
            return hidden
        return fwd

    def _checkpointed_forward(self, hidden, mask, enc_out, enc_dec_mask, position_ids):
        n = self.num_layers
        if self.recompute_method == "uniform":
            i = 0
            while i < n:
                hidden = tp.checkpoint(self._run(i, min(i + self.recompute_num_layers, n)),
                                       self.distribute_saved_activations, hidden, mask, enc_out,
                                       enc_dec_mask, position_ids)
                i += self.recompute_num_layers
        elif self.recompute_method == "block":
            for i in range(n):
                if i < self.recompute_num_layers:
                    hidden = tp.checkpoint(self._run(i, i + 1), self.distribute_saved_activations,
                                           hidden, mask, enc_out, enc_dec_mask, position_ids)
                else:
                    hidden = self._run(i, i + 1)(hidden, mask, enc_out, enc_dec_mask, position_ids)
        else:
            raise ValueError("Invalid activation recompute method.")
        return hidden

    def forward(self, hidden_states, attention_mask, encoder_output=None, enc_dec_attn_mask=None,
                inference_params=None, position_ids=None):
        if inference_params is not None and self.recompute_granularity is not None \
                and self.training:
            raise AssertionError("inference does not work with activation checkpointing")
        if not self.pre_process:
            hidden_states = self.input_tensor
        hidden_states = make_viewless_tensor(hidden_states, requires_grad=True, keep_graph=True)
        rng = tp.get_cuda_rng_tracker().fork() if self.sequence_parallel else nullcontext()
        with rng:
            if self.recompute_granularity == "full" and self.training:
                hidden_states = self._checkpointed_forward(hidden_states, attention_mask,
                                                           encoder_output, enc_dec_attn_mask,
                                                           position_ids)
            else:
                for layer in self.layers:
                    hidden_states = layer(hidden_states, attention_mask,
                                          encoder_output=encoder_output,
                                          enc_dec_attn_mask=enc_dec_attn_mask,
                                          inference_params=inference_params,
                                          position_ids=position_ids)
        if self.post_process and not self.use_post_ln:
            hidden_states = self.final_layernorm(hidden_states)
        return hidden_states
