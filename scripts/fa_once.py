"""Profiling driver: 5 FlashAttention forward launches at one shape
(default the 7B seq-1k shape b16 s1024 h32 hd128, causal), random bf16.

    python scripts/fa_once.py [b s nq nkv hd causal]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from epfl_megatron_amd.ops._ext import ext  # noqa: E402

b, s, nq, nkv, hd, causal = [int(v) for v in (sys.argv[1:7] if len(sys.argv) > 6
                                               else (16, 1024, 32, 32, 128, 1))]
C = ext()
q = torch.empty(b, s, nq, hd, device="cuda", dtype=torch.bfloat16).uniform_(-2, 2)
k = torch.empty(b, s, nkv, hd, device="cuda", dtype=torch.bfloat16).uniform_(-2, 2)
v = torch.empty(b, s, nkv, hd, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
out = torch.empty_like(q)
lse = torch.empty(b, nq, s, device="cuda", dtype=torch.float32)
r = nq // nkv
qs = [q.stride(0), q.stride(1), r * q.stride(2), q.stride(2)]
ks = [k.stride(0), k.stride(1), k.stride(2)]
for _ in range(5):
    C.flash_attn_fwd(q, k, v, out, lse, b, s, s, nq, nkv, hd, qs, ks, ks,
                     [out.stride(0), out.stride(1), out.stride(2)], bool(causal), hd ** -0.5,
                     None, None, None, None)
torch.cuda.synchronize()
print("done", flush=True)
