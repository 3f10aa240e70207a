"""Which FlashAttention forward / dQ kernels run on the Llama-2-70B TP8 rank's
attention shape, and its device time: first as the environment leaves it
(EMA_FA_KV2), then with the split-key forward switched on and off.

    python scripts/fa_kv2_probe.py
"""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from epfl_megatron_amd.ops._ext import ext
from epfl_megatron_amd.ops.attention import flash_attn_func
C = ext()
q = torch.randn(1, 4096, 8, 128, device="cuda", dtype=torch.bfloat16)
k = torch.randn(1, 4096, 1, 128, device="cuda", dtype=torch.bfloat16)
v = torch.randn_like(k)
for on in (None, True, False):
    if on is not None:
        C.fa_set_kv2(on)
    qq, kk, vv = (t.detach().requires_grad_() for t in (q, k, v))
    g = torch.randn_like(q)
    for _ in range(3):
        flash_attn_func(qq, kk, vv, causal=True).backward(g)
    torch.cuda.synchronize()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
        for _ in range(10):
            flash_attn_func(qq, kk, vv, causal=True).backward(g)
        torch.cuda.synchronize()
    for e in prof.key_averages():
        if "fa_fwd" in e.key or "fa_bwd_dq" in e.key:
            print(on, e.key[:90], e.count, round(e.device_time_total / max(1, e.count), 1), "us", flush=True)
C.fa_set_kv2(True)
