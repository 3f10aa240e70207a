"""Packed-document masks (--reset_attention_mask / --reset_position_ids) on CPU.

* the vectorised ``get_ltor_masks_and_position_ids`` against a loop oracle of
  the reference semantics (``megatron/utils.py:137-194``: for every EOD at j,
  rows > j stop seeing columns <= j, positions restart after j);
* the flash entry point with int32 document bounds (the form the HIP kernels
  take) against attention run on each document separately.
"""
import math

import torch

from epfl_megatron_amd.ops.attention import attention_ref, flash_attn_qkvpacked
from epfl_megatron_amd.utils.misc import doc_bounds, get_ltor_masks_and_position_ids


def _loop_oracle(data, eod):
    b, s = data.shape
    mask = torch.tril(torch.ones(b, s, s))
    pos = torch.arange(s).repeat(b, 1)
    for i in range(b):
        prev = 0
        for j in (data[i] == eod).nonzero().view(-1).tolist():
            mask[i, j + 1:, :j + 1] = 0
            pos[i, j + 1:] -= j + 1 - prev
            prev = j + 1
    return (mask < 0.5).unsqueeze(1), pos


def _tokens(b, s, seed):
    g = torch.Generator().manual_seed(seed)
    t = torch.randint(1, 50, (b, s), generator=g)
    t[torch.rand(b, s, generator=g) < 0.08] = 0
    t[0, -1] = 0  # EOD as the last token
    t[-1, 0] = 0  # EOD as the first token
    t[0, 5:7] = 0  # adjacent EODs
    return t


def test_masks_match_reference_loop():
    data = _tokens(3, 97, 0)
    m, lm, pos = get_ltor_masks_and_position_ids(data, 0, True, True, True)
    m_ref, pos_ref = _loop_oracle(data, 0)
    assert torch.equal(m, m_ref)
    assert torch.equal(pos, pos_ref)
    assert torch.equal(lm, (data != 0).float())
    # no reset: plain causal [1, 1, s, s], arange positions
    m2, _, pos2 = get_ltor_masks_and_position_ids(data, 0, False, False, False)
    assert m2.shape == (1, 1, 97, 97) and torch.equal(m2[0, 0], torch.triu(torch.ones(97, 97), 1).bool())
    assert torch.equal(pos2, torch.arange(97).expand(3, 97))


def test_doc_bounds_form():
    data = _tokens(2, 64, 1)
    bd, _, _ = get_ltor_masks_and_position_ids(data, 0, False, True, False, flash_doc_bounds=True)
    assert bd.dtype == torch.int32 and bd.shape == (2, 2, 64) and torch.equal(bd, doc_bounds(data, 0))
    start, end = bd[0].long(), bd[1].long()
    m_ref, _ = _loop_oracle(data, 0)
    j = torch.arange(64)
    for i in range(2):
        for q in range(64):
            seen = (~m_ref[i, 0, q]).nonzero().view(-1)
            assert seen.min() == start[i, q] and seen.max() == q
            # every position of q's document reports the same [start, end)
            assert (end[i, q] > q) and torch.all(start[i, start[i, q]:end[i, q]] == start[i, q])
    assert torch.all(end[:, :-1] <= 64)
    del j


def test_flash_entry_with_doc_bounds_equals_per_document_attention():
    torch.manual_seed(0)
    s, b, ng, r, hd = 80, 2, 2, 2, 16
    data = _tokens(b, s, 2)
    bd = doc_bounds(data, 0)
    qkv = torch.randn(s, b, ng * (r + 2) * hd)
    out = flash_attn_qkvpacked(qkv, ng, r, hd, causal=True, doc_bounds=bd)
    q5 = qkv.view(s, b, ng, r + 2, hd)
    q = q5[:, :, :, :r].reshape(s, b, ng * r, hd)
    k, v = q5[:, :, :, r], q5[:, :, :, r + 1]
    ref = torch.empty(s, b, ng * r, hd)
    for i in range(b):
        q0 = 0
        while q0 < s:
            q1 = int(bd[1, i, q0])
            o = attention_ref(q[q0:q1, i:i + 1].transpose(0, 1), k[q0:q1, i:i + 1].transpose(0, 1),
                              v[q0:q1, i:i + 1].transpose(0, 1), True, 1.0 / math.sqrt(hd))
            ref[q0:q1, i] = o[0]
            q0 = q1
    torch.testing.assert_close(out.view(s, b, ng * r, hd), ref, atol=1e-5, rtol=1e-5)
