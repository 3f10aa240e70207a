"""FlashAttention forward/backward timing on the training shapes (1 GPU).

Usage: python scripts/fa_bench2.py [b,s,nq,nkv,hd ...].  Median of 10 timed launches after 3 warm-up launches, random
data, causal; TF/s counts the causal half (4*b*nq*s^2*hd/2 fwd, 2.5x that bwd).
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from epfl_megatron_amd.ops.attention import flash_attn_func  # noqa: E402

SHAPES = ["16,1024,32,32,128", "4,4096,32,32,128", "8,2048,32,2,64", "2,4096,8,1,128"]


def bench(b, s, nq, nkv, hd):
    torch.manual_seed(0)
    q = torch.randn(b, s, nq, hd, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(b, s, nkv, hd, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(b, s, nkv, hd, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    do = torch.randn(b, s, nq, hd, device="cuda", dtype=torch.bfloat16)
    fl = 4.0 * b * nq * s * s * hd / 2
    tf, tb = [], []
    for it in range(13):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record()
        o = flash_attn_func(q, k, v, causal=True)
        e[1].record()
        o.backward(do)
        e[2].record()
        torch.cuda.synchronize()
        if it >= 3:
            tf.append(e[0].elapsed_time(e[1]))
            tb.append(e[1].elapsed_time(e[2]))
        q.grad = k.grad = v.grad = None
    mf, mb = statistics.median(tf), statistics.median(tb)
    print(f"shape={b},{s},{nq},{nkv},{hd}: "
          f"fwd {mf * 1e3:.1f} us {fl / mf / 1e9:.0f} TF/s | bwd {mb * 1e3:.1f} us "
          f"{2.5 * fl / mb / 1e9:.0f} TF/s", flush=True)


if __name__ == "__main__":
    for sh in (sys.argv[1:] or SHAPES):
        bench(*[int(x) for x in sh.split(",")])
