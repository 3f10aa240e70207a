"""Five causal forward calls at b=8 s=1024 nq=32 hd=128 (a short program for
rocprofv3 --pmc passes over the FlashAttention forward)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from epfl_megatron_amd.ops.attention import flash_attn_func  # noqa: E402

q = torch.randn(8, 1024, 32, 128, device="cuda", dtype=torch.bfloat16)
k, v = torch.randn_like(q), torch.randn_like(q)
with torch.no_grad():
    for _ in range(5):
        flash_attn_func(q, k, v, causal=True)
torch.cuda.synchronize()
print("ok")
