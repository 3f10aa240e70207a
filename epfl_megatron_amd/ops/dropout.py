"""Fused residual + dropout(x [+ x2] [+ bias]) (reference ``bias_dropout_add``,
``megatron/model/transformer.py:538-578``; TorchScript-fused there).

GPU: one HIP pass (``csrc/dropout.hip``).  The mask is counter-based
Philox-4x32-10 keyed by the current torch CUDA generator's (seed, offset); the
generator offset is advanced once per call, so the stream is reproducible
from the seed, moves with every other dropout, and — inside the
tensor-parallel RNG tracker's fork (sequence parallel) — differs per TP rank
exactly like the reference's.  Backward regenerates the mask: nothing is saved
but two integers.  ``philox_keep_mask`` is a NumPy transcription used by the
tests to check the GPU mask bit for bit.

CPU (gloo plumbing path): plain PyTorch ops with ``F.dropout``.
"""
import numpy as np
import torch
import torch.nn.functional as F

from ._ext import ext, use_native

_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
_MASK32 = np.uint64(0xFFFFFFFF)


def _philox(ctr, offset, seed):
    """Philox-4x32-10 of counter (ctr_lo, ctr_hi, off_lo, off_hi), key seed -> 4 x uint32."""
    ctr = ctr.astype(np.uint64)
    c0 = (ctr & _MASK32).astype(np.uint32)
    c1 = (ctr >> np.uint64(32)).astype(np.uint32)
    c2 = np.full_like(c0, np.uint32(offset & 0xFFFFFFFF))
    c3 = np.full_like(c0, np.uint32((offset >> 32) & 0xFFFFFFFF))
    k0, k1 = np.uint32(seed & 0xFFFFFFFF), np.uint32((seed >> 32) & 0xFFFFFFFF)
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = _M0 * c0.astype(np.uint64)
            p1 = _M1 * c2.astype(np.uint64)
            n0 = (p1 >> np.uint64(32)).astype(np.uint32) ^ c1 ^ k0
            n1 = (p1 & _MASK32).astype(np.uint32)
            n2 = (p0 >> np.uint64(32)).astype(np.uint32) ^ c3 ^ k1
            n3 = (p0 & _MASK32).astype(np.uint32)
            c0, c1, c2, c3 = n0, n1, n2, n3
            k0 = np.uint32((int(k0) + int(_W0)) & 0xFFFFFFFF)
            k1 = np.uint32((int(k1) + int(_W1)) & 0xFFFFFFFF)
    return c0, c1, c2, c3


def _threshold(p):
    return min(int(p * 4294967296.0), 4294967295) if p > 0 else 0


def philox_keep_mask(n, p, seed, offset):
    """The GPU kernel's keep-mask for a flat tensor of ``n`` elements (bool [n])."""
    nvec = n // 8
    idx = np.arange(nvec, dtype=np.uint64)
    a = _philox(2 * idx, offset, seed)
    b = _philox(2 * idx + 1, offset, seed)
    u = np.stack(list(a) + list(b), axis=1).reshape(-1)  # 8 uniforms per vector, in order
    return u >= np.uint32(_threshold(p))


def _next_philox(device):
    """(seed, offset) for one call; advances the generator past it."""
    gen = torch.cuda.default_generators[device.index if device.index is not None
                                        else torch.cuda.current_device()]
    seed = gen.initial_seed()
    offset = gen.get_offset()
    gen.set_offset(offset + 4)
    return seed, offset


class _FusedBDA(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, x2, bias, residual, p):
        seed, offset = _next_philox(x.device) if p > 0.0 else (0, 0)
        out = ext().bias_dropout_add_fwd(x.contiguous(), None if x2 is None else x2.contiguous(),
                                         bias, residual.contiguous(), p, seed, offset)
        ctx.p, ctx.seed, ctx.offset = p, seed, offset
        ctx.has_x2, ctx.has_bias = x2 is not None, bias is not None
        ctx.shape = x.shape
        return out

    @staticmethod
    def backward(ctx, dout):
        dout = dout.contiguous()
        dx = ext().bias_dropout_add_bwd(dout, ctx.p, ctx.seed, ctx.offset) if ctx.p > 0.0 \
            else dout
        dbias = dx.reshape(-1, dx.shape[-1]).float().sum(0).to(dx.dtype) if ctx.has_bias else None
        return dx, (dx if ctx.has_x2 else None), dbias, dout, None


def _supported(x, residual):
    return (use_native(x) and x.dtype in (torch.bfloat16, torch.float16)
            and residual.dtype == x.dtype and x.shape == residual.shape
            and x.shape[-1] % 8 == 0)


def bias_dropout_add(x, bias, residual, p, training, x2=None):
    """``residual + dropout(x [+ x2] [+ bias], p)`` (dropout only when training)."""
    p = float(p) if training else 0.0
    if _supported(x, residual) and (bias is None or bias.dtype == x.dtype) \
            and (x2 is None or x2.shape == x.shape):
        return _FusedBDA.apply(x, x2, bias, residual, p)
    y = x if x2 is None else x + x2
    if bias is not None:
        y = y + bias
    if p > 0.0:
        y = F.dropout(y, p=p, training=True)
    return residual + y
