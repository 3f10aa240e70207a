"""Decode-attention debug: which (batch, head, dim) elements differ from the reference."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from epfl_megatron_amd.ops.attention import attention_ref, _flash_decode  # noqa: E402

for (b, sk, nq, nkv, hd) in ((2, 1, 8, 8, 128), (2, 77, 8, 8, 128), (1, 300, 8, 8, 128), (2, 77, 8, 2, 128)):
    torch.manual_seed(0)
    kmem = torch.randn(sk + 5, b + 1, nkv, hd, device="cuda", dtype=torch.bfloat16)
    vmem = torch.randn(sk + 5, b + 1, nkv, hd, device="cuda", dtype=torch.bfloat16)
    q = torch.randn(1, b, nq, hd, device="cuda", dtype=torch.bfloat16) * 2
    keys, vals = kmem[:sk, 1:b + 1].transpose(0, 1), vmem[:sk, 1:b + 1].transpose(0, 1)
    o = _flash_decode(q.transpose(0, 1), keys, vals, hd ** -0.5)
    orf = attention_ref(q.transpose(0, 1).float(), keys.float(), vals.float(), causal=True)
    err = (o.float() - orf).abs()[:, 0]  # [b, nq, hd]
    bad = err > 0.05
    print((b, sk, nq, nkv, hd), "bad", int(bad.sum()), "per batch", bad.sum((1, 2)).tolist(),
          "per head", bad.sum((0, 2)).tolist(), "dims even/odd", int(bad[..., 0::2].sum()), int(bad[..., 1::2].sum()),
          "first dims", bad.sum((0, 1))[:8].tolist(), "max", float(err.max()))
    if sk == 1:
        print(" o[0,0,:6]", o[0, 0, 0, :6].float().tolist(), " ref", orf[0, 0, 0, :6].tolist())
