"""Fused QKV layout helpers (reference ``weights2megatron/permute_qkv.py``,
``weights2megatron/weights2megatron.py:87-99``, ``megatron2hf.py:60-84``).

Megatron's fused QKV weight is grouped per KV head::

    rows = [ q_0 .. q_{r-1}, k, v ]  for each of the n_kv groups   (r = n_heads / n_kv)

each block being ``head_dim`` rows.  RoPE here rotates interleaved pairs
``(2i, 2i+1)`` (Meta convention), while Hugging Face checkpoints rotate
``(i, i + head_dim/2)`` ("rotate_half"); converting between the two is a
fixed row permutation inside every q and k head block, v untouched.
"""
import torch


def _head_perm(head_dim, to_interleaved):
    """Row order that maps a rotate-half head block to interleaved (or back)."""
    half = head_dim // 2
    idx = torch.arange(head_dim)
    if to_interleaved:  # new row 2i <- old i, new row 2i+1 <- old i+half
        return torch.stack((idx[:half], idx[half:]), dim=1).reshape(-1)
    return torch.cat((idx[0::2], idx[1::2]))


def permute_qkv(qkv_w, dim, n_heads, n_heads_kv, revert=False):
    """HF rotate-half rows -> interleaved rows of every q/k head (``revert``: back).

    Works on a fused grouped QKV weight (or bias, 1-D) with ``dim // n_heads``
    rows per head; returns a new tensor.
    """
    head_dim = dim // n_heads
    r = n_heads // n_heads_kv
    n_groups = qkv_w.shape[0] // (head_dim * (r + 2))
    perm = _head_perm(head_dim, to_interleaved=not revert)
    rows = []
    for g in range(n_groups):
        for j in range(r + 2):
            base = (g * (r + 2) + j) * head_dim
            block = torch.arange(base, base + head_dim)
            rows.append(block if j == r + 1 else block[perm])
    return qkv_w.index_select(0, torch.cat(rows).to(qkv_w.device))


def pack_qkv(wq, wk, wv, n_heads, n_heads_kv):
    """Separate q ``[nq*hd, h]``, k/v ``[nkv*hd, h]`` -> grouped fused QKV."""
    hd = wq.shape[0] // n_heads
    r = n_heads // n_heads_kv
    q = wq.reshape(n_heads_kv, r * hd, *wq.shape[1:])
    k = wk.reshape(n_heads_kv, hd, *wk.shape[1:])
    v = wv.reshape(n_heads_kv, hd, *wv.shape[1:])
    return torch.cat((q, k, v), dim=1).reshape(-1, *wq.shape[1:])


def unpack_qkv(qkv, n_heads, n_heads_kv, head_dim):
    """Grouped fused QKV -> (wq, wk, wv)."""
    r = n_heads // n_heads_kv
    g = qkv.reshape(n_heads_kv, (r + 2) * head_dim, *qkv.shape[1:])
    wq = g[:, :r * head_dim].reshape(-1, *qkv.shape[1:])
    wk = g[:, r * head_dim:(r + 1) * head_dim].reshape(-1, *qkv.shape[1:])
    wv = g[:, (r + 1) * head_dim:].reshape(-1, *qkv.shape[1:])
    return wq.contiguous(), wk.contiguous(), wv.contiguous()
