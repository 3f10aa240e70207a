"""Fused attention.

``flash_attn_qkvpacked`` is the training hot path: it takes the fused QKV
projection output in the reference's GQA layout ``[s, b, ng, r+2, hd]``
(r = nq/nkv query heads per KV group, then k, then v;
reference ``megatron/model/transformer.py:445-455``) and runs the
hand-written gfx950 FlashAttention-2 kernel
(``csrc/flash_attn_fwd.hip`` / ``flash_attn_bwd.hip``) reading Q/K/V through
strides.  GQA/MQA is native: query head ``j`` reads KV group ``j // r``; K/V
are never expanded to ``nq`` heads (the reference broadcast them, D2).
RoPE is fused: a k-only pass rotates the key heads, the forward kernel
rotates Q in registers (and writes it back for the backward), and the
backward kernels apply R^T to dQ/dK in their epilogues while writing them
straight into a ``[s, b, ng, r+2, hd]`` gradient buffer for the QKV GEMM
backward.

``flash_attn_func`` is the general entry (separate q/k/v, ``sq <= sk`` with
bottom-right-aligned causal mask) used by KV-cached inference; single-token
decode steps go to the split-key decode kernel (``csrc/flash_decode.hip``).

CPU tensors use an exact fp32 math reference (GPU test oracle and the gloo
plumbing path).
"""
import math

import torch

from ._ext import ext, use_native
from .rope import rope_qkv_inplace, apply_rope_ref


# --------------------------------------------------------------------------
# Reference math (CPU path + test oracle)
# --------------------------------------------------------------------------
def attention_ref(q, k, v, causal=True, softmax_scale=None, return_lse=False, doc_bounds=None):
    """q ``[b, sq, nq, d]``, k/v ``[b, sk, nkv, d]`` -> ``[b, sq, nq, d]`` (fp32 math).

    ``doc_bounds``: optional int32 ``[2, b, s]`` (document start, end) of
    packed sequences: query i sees key j only if ``doc_start[i] <= j``."""
    b, sq, nq, d = q.shape
    sk, nkv = k.shape[1], k.shape[2]
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(d)
    rep = nq // nkv
    qf = q.float().permute(0, 2, 1, 3)
    kf = k.float().permute(0, 2, 1, 3).repeat_interleave(rep, dim=1)
    vf = v.float().permute(0, 2, 1, 3).repeat_interleave(rep, dim=1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:
        i = torch.arange(sq, device=q.device)[:, None]
        j = torch.arange(sk, device=q.device)[None, :]
        s = s.masked_fill(j > i + (sk - sq), float("-inf"))
    if doc_bounds is not None:
        j = torch.arange(sk, device=q.device)[None, None, :]
        before = j < doc_bounds[0].to(q.device).long()[:, :, None]  # [b, sq, sk]
        s = s.masked_fill(before[:, None], float("-inf"))
    lse = torch.logsumexp(s, dim=-1)
    p = torch.softmax(s, dim=-1)
    o = torch.matmul(p, vf).permute(0, 2, 1, 3).to(q.dtype)
    if return_lse:
        return o, lse
    return o


def _split_qkv5(qkv5):
    s, b, ng, r2, hd = qkv5.shape
    r = r2 - 2
    q = qkv5[:, :, :, :r, :].reshape(s, b, ng * r, hd)
    k = qkv5[:, :, :, r, :]
    v = qkv5[:, :, :, r + 1, :]
    return q, k, v


# --------------------------------------------------------------------------
# Native path
# --------------------------------------------------------------------------
# One kernel signature serves every layout: each operand is a (tensor view,
# strides) pair.  Query head j lives at (j // r) * q_sg + (j % r) * q_sh and
# reads KV group j // r at g * k_sg; all strides are in elements.
def _qkv5_views(qkv5):
    s, b, ng, r2, hd = qkv5.shape
    r = r2 - 2
    ss, sb, sg, sh, sd = qkv5.stride()
    if sd != 1:
        raise AssertionError("head_dim must be contiguous")
    q = qkv5[:, :, :, 0, :]
    k = qkv5[:, :, :, r, :]
    v = qkv5[:, :, :, r + 1, :]
    qs = (sb, ss, sg, sh)
    ks = (sb, ss, sg)
    return q, k, v, qs, ks


def _bsnd_strides(t, r):
    """[b, s, n, d] tensor -> (sb, ss, sg, sh) with group stride r*sh."""
    sb, ss, sh, sd = t.stride()
    if sd != 1:
        raise AssertionError("head_dim must be contiguous")
    return (sb, ss, r * sh, sh)


class _FlashQKVPackedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, ng, r, hd, causal, scale, cos, sin, position_ids, docs):
        s, b = qkv.shape[0], qkv.shape[1]
        qkv5 = qkv.view(s, b, ng, r + 2, hd)
        if position_ids is not None and position_ids.dtype != torch.int64:
            position_ids = position_ids.long()
        if cos is not None:  # keys only: Q is rotated inside the attention kernel
            rope_qkv_inplace(qkv5, cos, sin, position_ids, k_only=True)
        q, k, v, qs, ks = _qkv5_views(qkv5)
        nq = ng * r
        out = torch.empty(s, b, nq, hd, dtype=qkv.dtype, device=qkv.device)
        lse = torch.empty(b, nq, s, dtype=torch.float32, device=qkv.device)
        os_ = (out.stride(1), out.stride(0), out.stride(2))
        ext().flash_attn_fwd(q, k, v, out, lse, b, s, s, nq, ng, hd,
                             list(qs), list(ks), list(ks), list(os_), bool(causal), float(scale),
                             cos, sin, position_ids, docs)
        ctx.save_for_backward(qkv, out, lse, cos, sin, position_ids, docs)
        ctx.meta = (ng, r, hd, causal, scale)
        return out.view(s, b, nq * hd)

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse, cos, sin, position_ids, docs = ctx.saved_tensors
        ng, r, hd, causal, scale = ctx.meta
        s, b = qkv.shape[0], qkv.shape[1]
        nq = ng * r
        qkv5 = qkv.view(s, b, ng, r + 2, hd)
        dout = dout.reshape(s, b, nq, hd)
        if not dout.is_contiguous():
            dout = dout.contiguous()
        dqkv5 = torch.empty_like(qkv5)
        q, k, v, qs, ks = _qkv5_views(qkv5)
        dq, dk, dv, _, _ = _qkv5_views(dqkv5)
        os_ = (out.stride(1), out.stride(0), out.stride(2))
        ext().flash_attn_bwd(dout, q, k, v, out, lse, dq, dk, dv, b, s, s, nq, ng, hd,
                             list(qs), list(ks), list(ks), list(os_), bool(causal), float(scale),
                             cos, sin, position_ids, docs)
        return dqkv5.view(s, b, -1), None, None, None, None, None, None, None, None, None


def _flash_decode(q, k, v, scale, kv_len=None):
    """sq == 1 against a KV cache (generation): split-key decode kernel
    (``csrc/flash_decode.hip``); no autograd.  ``kv_len``: optional device
    int32 tensor with the number of valid keys (k / v then span the whole
    cache; the launch does not depend on the step, for hipGraph capture)."""
    b, _, nq, d = q.shape
    sk, nkv = k.shape[1], k.shape[2]
    r = nq // nkv
    out = torch.empty(b, 1, nq, d, dtype=q.dtype, device=q.device)
    ext().flash_decode(q, k, v, out, b, sk, nq, nkv, d, list(_bsnd_strides(q, r)),
                       list(_bsnd_strides(k, 1)[:3]), list(_bsnd_strides(v, 1)[:3]),
                       [out.stride(0), out.stride(1), out.stride(2)], float(scale), kv_len)
    return out


def flash_decode_cached(q, k, v, kv_len, softmax_scale=None):
    """One query row per sequence against a whole KV cache ``k / v [b, smax,
    nkv, d]`` of which the first ``kv_len`` (device int32) keys are valid."""
    if not use_native(q):
        n = int(kv_len.reshape(-1)[0])
        return attention_ref(q, k[:, :n], v[:, :n], False,
                             softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(q.shape[-1]))
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(q.shape[-1])
    return _flash_decode(q, k, v, scale, kv_len)


class _FlashFn(torch.autograd.Function):
    """Separate q ``[b, sq, nq, d]``, k/v ``[b, sk, nkv, d]``."""

    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        b, sq, nq, d = q.shape
        sk, nkv = k.shape[1], k.shape[2]
        r = nq // nkv
        out = torch.empty(b, sq, nq, d, dtype=q.dtype, device=q.device)
        lse = torch.empty(b, nq, sq, dtype=torch.float32, device=q.device)
        qs = _bsnd_strides(q, r)
        ks = _bsnd_strides(k, 1)[:3]
        vs = _bsnd_strides(v, 1)[:3]
        os_ = (out.stride(0), out.stride(1), out.stride(2))
        ext().flash_attn_fwd(q, k, v, out, lse, b, sq, sk, nq, nkv, d,
                             list(qs), list(ks), list(vs), list(os_), bool(causal), float(scale),
                             None, None, None, None)
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.causal, ctx.scale = causal, scale
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, out, lse = ctx.saved_tensors
        b, sq, nq, d = q.shape
        sk, nkv = k.shape[1], k.shape[2]
        r = nq // nkv
        dout = dout.contiguous()
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        qs = _bsnd_strides(q, r)
        ks = _bsnd_strides(k, 1)[:3]
        os_ = (out.stride(0), out.stride(1), out.stride(2))
        ext().flash_attn_bwd(dout, q, k, v, out, lse, dq, dk, dv, b, sq, sk, nq, nkv, d,
                             list(qs), list(ks), list(ks), list(os_), bool(ctx.causal),
                             float(ctx.scale), None, None, None, None)
        return dq, dk, dv, None, None


def flash_attn_qkvpacked(qkv, num_groups, q_per_group, head_dim, causal=True,
                         softmax_scale=None, rope=None, position_ids=None, doc_bounds=None):
    """qkv ``[s, b, ng*(r+2)*hd]`` -> context ``[s, b, ng*r*hd]``.

    ``rope`` = (cos, sin) tables or None.  ``doc_bounds``: int32 ``[2, b, s]``
    document (start, end) per position for packed sequences
    (``--reset_attention_mask``; :func:`utils.misc.doc_bounds`), or None."""
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(head_dim)
    cos, sin = rope if rope is not None else (None, None)
    if doc_bounds is not None:
        if not causal:
            raise ValueError("document masking is defined for causal attention only")
        doc_bounds = doc_bounds.to(device=qkv.device, dtype=torch.int32).contiguous()
    if use_native(qkv):
        return _FlashQKVPackedFn.apply(qkv, num_groups, q_per_group, head_dim, causal, scale,
                                       cos, sin, position_ids, doc_bounds)
    s, b = qkv.shape[0], qkv.shape[1]
    qkv5 = qkv.view(s, b, num_groups, q_per_group + 2, head_dim)
    q, k, v = _split_qkv5(qkv5)
    if cos is not None:
        q = apply_rope_ref(q, cos, sin, position_ids)
        k = apply_rope_ref(k, cos, sin, position_ids)
    o = attention_ref(q.transpose(0, 1), k.transpose(0, 1), v.transpose(0, 1), causal, scale,
                      doc_bounds=doc_bounds)
    return o.transpose(0, 1).reshape(s, b, -1)


def flash_attn_func(q, k, v, causal=True, softmax_scale=None):
    """Separate tensors ``[b, s, n, d]`` (inference / generic callers)."""
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if use_native(q):
        b, sq, nq = q.shape[:3]
        r = nq // k.shape[2]
        if sq == 1 and (r >= 2 or nq * b < 256 or k.shape[1] <= 512) and not (
                torch.is_grad_enabled() and (q.requires_grad or k.requires_grad or v.requires_grad)):
            # split-key decode: GQA/MQA reads each K/V byte once; small grids
            # spread over the chunks; short caches (profiles/r2f_decode_bench.txt)
            return _flash_decode(q, k, v, scale)  # the last position sees every cached key
        return _FlashFn.apply(q, k, v, causal, scale)
    return attention_ref(q, k, v, causal, scale)
