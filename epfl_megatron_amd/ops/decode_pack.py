"""Decode-packed weight layout for the weight-streaming skinny GEMM.

A decode step multiplies <= 32 rows by every weight of the model, so its time
is the weight stream from HBM (reference: ``megatron/text_generation/
generation.py:179-264`` runs the same step through the training GEMMs).  The
skinny kernel (``csrc/skinny_gemm.hip``) feeds ``v_mfma_f32_16x16x32`` with
lane L holding 8 consecutive k of W row ``L & 15``: on a row-major ``[N, K]``
weight one wave-load touches 16 rows x 64 B (every 4-lane quad four cache
lines) and the stream tops out at 3.9-4.9 TB/s.  ``pack`` reorders W so that
the fragments one wave loads for one k-step are a contiguous 1 KiB piece
(lane L at byte 16 L); the kernel's MFMA schedule and the k index each lane
feeds are unchanged, and the stream reaches 4.6-6.0 TB/s
(``scripts/gemv_layout_bench.hip``, ``profiles/r4m_gemv_layout.txt``).

Layout (K % 256 == 0, S = K / 256 k-steps of 32 per wave, 8 waves):
``packed[b, wave, s, q, r, e] = W[row(b, r), wave * 32 S + 32 s + 8 q + e]``
with ``row(b, r) = 16 b + r`` (plain / QKV) or, for a GLU weight ``[2F, K]``,
``8 b + r`` (up) / ``F + 8 b + r - 8`` (gate) — the kernel's ``w_row``.  The
last ``half_tail`` GLU blocks (``skinny_glu_half_tail``: the persistent
kernel's last round, run as twice as many 4-feature half units) follow as half
units ``[unit, wave, s, q, pr, e]`` (512 B per k-step) with ``pr`` = the 4 up
then the 4 gate rows of features ``8 b + 4 h .. + 3``; MFMA rows r and r + 4
of a half unit read the same bytes.

The packed copies live next to the parameter (``_ema_decode_packed``, one per
(GLU, half-tail) form, so the <= 16-row and 17-32-row decode forms do not
evict each other) and are rebuilt when the parameter's storage, in-place
version or the global weight generation changes.  The generation is bumped
by every optimizer step and checkpoint load (:func:`bump_weight_generation`):
those rewrite the weights through the DDP flat buffers, which does not move
the Parameter's ``_version``.  288 GB of HBM holds both layouts of a 70B TP8
shard many times over.  ``EMA_SKINNY_PACK=0`` streams the row-major
weights instead (A/B).
"""
import os

import torch

ENABLED = os.environ.get("EMA_SKINNY_PACK", "1") != "0"
_WEIGHT_GEN = [0]


def bump_weight_generation():
    """Weights may have been rewritten outside the Parameter objects
    (optimizer step, checkpoint load): every packed copy is stale."""
    _WEIGHT_GEN[0] += 1


def weight_generation():
    return _WEIGHT_GEN[0]


def packable(w):
    """W [N, K] the packed 8-wave skinny forms can read."""
    return (w.dim() == 2 and w.shape[1] % 256 == 0 and w.shape[0] % 16 == 0
            and w.dtype in (torch.bfloat16, torch.float16))


def pack(w, glu=False, half_tail=0):
    """The packed copy of ``w`` ([N, K] -> [N, K], same dtype / device)."""
    assert packable(w), f"skinny pack: unsupported weight {tuple(w.shape)} {w.dtype}"
    assert glu or not half_tail
    n, k = w.shape
    s = k // 256
    if glu:
        f = n // 2
        blocks = torch.stack((w[:f].reshape(f // 8, 8, k), w[f:].reshape(f // 8, 8, k)), 1)
        blocks = blocks.reshape(f // 8, 16, k)
    else:
        blocks = w.reshape(n // 16, 16, k)
    nb = blocks.shape[0]
    full = nb - half_tail
    # [b, r, wave, s, q, e] -> [b, wave, s, q, r, e]: lane q * 16 + r
    out = [blocks[:full].reshape(full, 16, 8, s, 4, 8).permute(0, 2, 3, 4, 1, 5).reshape(-1)]
    if half_tail:
        t = blocks[full:].reshape(half_tail, 2, 2, 4, k)  # [b, up|gate, h, row, k]
        t = t.permute(0, 2, 1, 3, 4).reshape(half_tail, 2, 8, 8, s, 4, 8)  # [b, h, pr, ...]
        # [b, h, pr, wave, s, q, e] -> [b, h, wave, s, q, pr, e]
        out.append(t.permute(0, 1, 3, 4, 5, 2, 6).reshape(-1))
    return torch.cat(out).reshape(n, k) if half_tail else out[0].reshape(n, k)


def unpack(p, glu=False, half_tail=0):
    """Inverse of ``pack`` (tests)."""
    n, k = p.shape
    s = k // 256
    nb = n // 16
    full = nb - half_tail
    flat = p.reshape(-1)
    blocks = flat[:full * 16 * k].reshape(full, 8, s, 4, 16, 8).permute(0, 4, 1, 2, 3, 5)
    blocks = [blocks.reshape(full, 16, k)]
    if half_tail:
        t = flat[full * 16 * k:].reshape(half_tail, 2, 8, s, 4, 8, 8).permute(0, 1, 5, 2, 3, 4, 6)
        t = t.reshape(half_tail, 2, 2, 4, k).permute(0, 2, 1, 3, 4)  # [b, up|gate, h, row, k]
        blocks.append(t.reshape(half_tail, 16, k))
    blocks = torch.cat(blocks)
    if glu:
        f = n // 2
        return torch.cat((blocks[:, :8].reshape(f, k), blocks[:, 8:].reshape(f, k)), 0)
    return blocks.reshape(n, k)


def packed(w, glu=False, half_tail=0):
    """Cached packed copy of parameter ``w``, or None when the row-major
    weight must be streamed (disabled / unsupported shape)."""
    if not ENABLED or not packable(w):
        return None
    form = (bool(glu), int(half_tail))
    key = (w.data_ptr(), w._version, _WEIGHT_GEN[0], w.dtype, tuple(w.shape))
    cache = getattr(w, "_ema_decode_packed", None)
    if not isinstance(cache, dict):
        cache = {}
        w._ema_decode_packed = cache
    hit = cache.get(form)
    if hit is not None and hit[0] == key:
        return hit[1]
    for f in [f for f, v in cache.items() if v[0] != key]:
        del cache[f]  # stale forms of an older generation
    with torch.no_grad():
        p = pack(w.detach(), glu, half_tail)
    cache[form] = (key, p)
    return p
