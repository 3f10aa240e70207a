"""Rotary position embeddings (Meta-Llama interleaved-pair convention).

Pairs are ``(x[2i], x[2i+1])`` rotated as complex numbers in fp32
(reference ``megatron/model/positional_embeddings.py:7-51``), with
``freq_i = theta^(-2i/d)`` and positions divided by ``rope_scaling_factor``.

MI355X design: the cos/sin table is built once per (dim, length, scaling,
device) and kept resident in HBM (the reference rebuilt it on the CPU and
copied it every forward).  On the GPU the rotation is applied by
a HIP kernel **in place** on the fused ``[s, b, ng, r+2, hd]`` QKV tensor that
the attention kernel then reads with strides — no rearrange/contiguous copies.
"""
import functools

import torch

from ._ext import ext, use_native


def precompute_freqs(dim, end, theta=10000.0, scaling_factor=1.0):
    """fp32 angles ``[end, dim/2]`` (same arithmetic as the reference table)."""
    inv = 1.0 / (theta ** (torch.arange(0, dim, 2).float() / dim))
    t = torch.arange(end).float() / scaling_factor
    return torch.outer(t, inv).float()


@functools.lru_cache(maxsize=32)
def _rope_table_cached(dim, end, theta, scaling_factor, device):
    ang = precompute_freqs(dim, end, theta, scaling_factor)
    cos = torch.cos(ang)
    sin = torch.sin(ang)
    if device != "cpu":
        cos, sin = cos.to(device), sin.to(device)
    return cos.contiguous(), sin.contiguous()


def rope_table(dim, end, device, theta=10000.0, scaling_factor=1.0):
    dev = str(torch.device(device)) if not isinstance(device, str) else device
    if dev.startswith("cuda") and ":" not in dev:
        dev = f"cuda:{torch.cuda.current_device()}"
    return _rope_table_cached(dim, end, float(theta), float(scaling_factor), dev)


def apply_rope_ref(x, cos, sin, position_ids=None, offset=0, inverse=False):
    """x: ``[s, b, n, d]`` (any dtype).  Rotates interleaved pairs in fp32.

    position_ids: ``[b, s]`` or None (=> ``offset + arange(s)``)."""
    s, b = x.shape[0], x.shape[1]
    if position_ids is None:
        pos = torch.arange(offset, offset + s, device=x.device)
        c = cos[pos][:, None, None, :]
        sn = sin[pos][:, None, None, :]
    else:
        pos = position_ids.to(x.device).t()  # [s, b]
        c = cos[pos][:, :, None, :]
        sn = sin[pos][:, :, None, :]
    if inverse:
        sn = -sn
    xf = x.float().reshape(*x.shape[:-1], -1, 2)
    x0, x1 = xf[..., 0], xf[..., 1]
    out = torch.stack((x0 * c - x1 * sn, x0 * sn + x1 * c), dim=-1).flatten(-2)
    return out.type_as(x)


def rope_qkv_inplace(qkv5, cos, sin, position_ids=None, offset=0, inverse=False,
                     k_only=False):
    """Rotate q and k heads (``k_only``: just the key heads) of a fused
    ``[s, b, ng, r+2, hd]`` tensor in place.

    Not an autograd op: callers (the attention Function) own the gradient."""
    if use_native(qkv5):
        pos = position_ids
        if pos is not None and pos.dtype != torch.int64:
            pos = pos.long()
        ext().rope_qkv_inplace(qkv5, cos, sin, pos, int(offset), bool(inverse), bool(k_only))
        return qkv5
    r2 = qkv5.shape[3]
    s, b, ng, _, hd = qkv5.shape
    lo = r2 - 2 if k_only else 0
    qk = qkv5[:, :, :, lo:r2 - 1, :].reshape(s, b, ng * (r2 - 1 - lo), hd)
    rot = apply_rope_ref(qk, cos, sin, position_ids, offset, inverse)
    qkv5[:, :, :, lo:r2 - 1, :].copy_(rot.view(s, b, ng, r2 - 1 - lo, hd))
    return qkv5


class _RopeQKVFn(torch.autograd.Function):
    """Out-of-place rotation of the q and k heads of ``[s, b, ng, r+2, hd]``;
    the backward rotates the gradient back (R^T), v passes through."""

    @staticmethod
    def forward(ctx, qkv5, cos, sin, position_ids):
        ctx.save_for_backward(cos, sin, position_ids)
        return rope_qkv_inplace(qkv5.contiguous().clone(), cos, sin, position_ids)

    @staticmethod
    def backward(ctx, g):
        cos, sin, position_ids = ctx.saved_tensors
        return rope_qkv_inplace(g.contiguous().clone(), cos, sin, position_ids,
                                inverse=True), None, None, None


def rope_qkv(qkv5, cos, sin, position_ids):
    """Autograd form of ``rope_qkv_inplace`` (HIP kernel on the GPU)."""
    return _RopeQKVFn.apply(qkv5, cos, sin, position_ids)


def apply_rotary_emb(xq, xk, cos, sin, position_ids=None, offset=0):
    """Out-of-place rotation of separate q ``[s,b,nq,d]`` and k ``[s,b,nk,d]``."""
    return (apply_rope_ref(xq, cos, sin, position_ids, offset),
            apply_rope_ref(xk, cos, sin, position_ids, offset))
