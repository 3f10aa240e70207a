"""Flat-buffer optimizer kernels.

The optimizer state of the whole model is held in flat fp32 buffers laid out
like the DDP gradient buffer, so the update is ONE streaming pass
(``csrc/optim.hip``) over ``(grad, master, m, v) -> (master, m, v, bf16 param)``
instead of apex's multi-tensor-apply over hundreds of tensor lists.  A static
chunk table (built once, device resident) maps chunks of the master buffer to
their gradient/param offsets, param group (lr/wd) and whether the chunk counts
toward the global grad norm (TP duplicates and shared params do not).

Chunk table: int64 ``[n, 4]`` = (master_off, buf_off, length, meta) with
``meta = group | (count_in_norm << 8)``.
"""
import math

import torch

from ._ext import ext, use_native

CHUNK = 1 << 16


class ChunkPlan:
    """Static description of the flat optimizer layout.

    ``rows``: coarse python list of (master_off, buf_off, length, meta) segments
    (used by torch loops); ``table``: the same cut into CHUNK-element rows as a
    device int64 tensor (one workgroup per row in the HIP kernels)."""

    def __init__(self, segments, device):
        self.rows = []
        for m_off, b_off, n, g, cnt in segments:
            if n > 0:
                self.rows.append((m_off, b_off, n, int(g) | (int(bool(cnt)) << 8)))
        fine = []
        for m_off, b_off, n, meta in self.rows:
            for st in range(0, n, CHUNK):
                fine.append((m_off + st, b_off + st, min(CHUNK, n - st), meta))
        if not fine:
            fine = [(0, 0, 0, 0)]
        self.table = torch.tensor(fine, dtype=torch.int64, device=device) \
            if str(device).startswith("cuda") else None


def grad_norm_sq(grad_buf, plan):
    """Sum of squares of the gradient chunks flagged ``count_in_norm`` (fp32 scalar)."""
    if use_native(grad_buf):
        return ext().chunked_sumsq(grad_buf, plan.table)
    total = torch.zeros((), dtype=torch.float32, device=grad_buf.device)
    for m_off, b_off, n, meta in plan.rows:
        if meta >> 8:
            total += grad_buf[b_off:b_off + n].float().pow(2).sum()
    return total


def count_zeros(grad_buf, plan):
    total = 0
    for m_off, b_off, n, meta in plan.rows:
        if meta >> 8:
            total += int((grad_buf[b_off:b_off + n] == 0).sum().item())
    return total


def step_prep(norm_sq, inv_scale, clip, st):
    """Device epilogue of the grad-norm reduction (no host sync):
    ``st`` (fp32 [4]) <- [scale = clip_coef * inv_scale, found_inf, step (+1 unless
    found_inf), grad_norm].  Reference semantics: ``optimizer.py:408-466`` (skip on
    a non-finite norm, EPFL addition :442-444) and ``clip_grads.py:16-107``."""
    if use_native(st):
        ext().opt_prep(norm_sq.reshape(1).float(), inv_scale, float(clip), st)
        return st
    raw = norm_sq.reshape(()).float()
    bad = ~torch.isfinite(raw)
    inv = inv_scale.reshape(()).float() if inv_scale is not None else torch.ones_like(raw)
    gn = torch.sqrt(raw) * inv
    coef = torch.ones_like(raw)
    if clip > 0.0:
        coef = torch.clamp(clip / (gn + 1.0e-6), max=1.0)
    st[0] = torch.where(bad, torch.zeros_like(raw), coef * inv)
    st[1] = bad.float()
    st[2] = st[2] + (~bad).float()
    st[3] = torch.where(bad, torch.full_like(raw, float("nan")), gn)
    return st


def adam_step(master, model_out, grad_buf, exp_avg, exp_avg_sq, plan, lrs, wds, beta1, beta2,
              eps, step, grad_scale, adam_w_mode=True, dev_state=None):
    """Fused AdamW over all chunks (apex FusedAdam math, bias correction on).

    ``grad_scale`` multiplies the gradient first (clip coef x 1/loss-scale).
    ``model_out`` (bf16/fp16 param buffer, same layout as ``grad_buf``) gets the
    updated params in the same pass; None when master *is* the param buffer.
    ``dev_state`` (from ``step_prep``) replaces ``grad_scale`` / ``step`` with
    device values and makes the update a no-op when the norm was non-finite."""
    if use_native(master):
        bc1 = 1.0 - beta1 ** max(step, 1)
        bc2 = 1.0 - beta2 ** max(step, 1)
        ext().flat_adam(master, model_out, grad_buf, exp_avg, exp_avg_sq, plan.table,
                        [float(x) for x in lrs], [float(x) for x in wds], float(beta1),
                        float(beta2), float(eps), float(bc1), float(bc2), float(grad_scale),
                        bool(adam_w_mode), dev_state)
        return
    if dev_state is not None:
        # CPU path: reading the device state is free (no GPU queue to drain)
        if float(dev_state[1]) != 0.0:
            return
        grad_scale = float(dev_state[0])
        step = int(round(float(dev_state[2])))
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    for m_off, b_off, n, meta in plan.rows:
        if n == 0:
            continue
        g_idx = meta & 0xFF
        lr, wd = lrs[g_idx], wds[g_idx]
        p = master[m_off:m_off + n]
        g = grad_buf[b_off:b_off + n].float() * grad_scale
        m = exp_avg[m_off:m_off + n]
        v = exp_avg_sq[m_off:m_off + n]
        if not adam_w_mode:
            g = g + wd * p
        m.mul_(beta1).add_(g, alpha=1 - beta1)
        v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
        denom = (v / bc2).sqrt_().add_(eps)
        upd = (m / bc1) / denom
        if adam_w_mode:
            upd = upd + wd * p
        p.add_(upd, alpha=-lr)
        if model_out is not None:
            model_out[b_off:b_off + n].copy_(p)


def sgd_step(master, model_out, grad_buf, momentum_buf, plan, lrs, wds, momentum, grad_scale,
             dev_state=None):
    """SGD with momentum (apex FusedSGD semantics: wd added to the grad).
    With ``dev_state`` the scale is a device scalar and a skipped step is
    masked on the device (no host sync)."""
    skip = None
    if dev_state is not None:
        grad_scale = dev_state[0]
        skip = dev_state[1] != 0
    for m_off, b_off, n, meta in plan.rows:
        if n == 0:
            continue
        g_idx = meta & 0xFF
        lr, wd = lrs[g_idx], wds[g_idx]
        p = master[m_off:m_off + n]
        g = grad_buf[b_off:b_off + n].float() * grad_scale + wd * p
        if momentum > 0:
            buf = momentum_buf[m_off:m_off + n]
            if skip is not None:
                buf.copy_(torch.where(skip, buf, buf * momentum + g))
            else:
                buf.mul_(momentum).add_(g)
            g = buf
        if skip is not None:
            p.copy_(torch.where(skip, p, p - lr * g))
        else:
            p.add_(g, alpha=-lr)
        if model_out is not None:
            model_out[b_off:b_off + n].copy_(p)


def copy_master_to_model(master, model_out, plan):
    for m_off, b_off, n, meta in plan.rows:
        if n:
            model_out[b_off:b_off + n].copy_(master[m_off:m_off + n])
