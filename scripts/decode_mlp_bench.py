"""Fused decode MLP (one persistent launch, grid barriers) vs the three skinny
launches, Llama-2-7B shapes.  python scripts/decode_mlp_bench.py"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from epfl_megatron_amd.ops._ext import ext  # noqa: E402


def t(fn, n=50):
    ts = []
    for it in range(n + 5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        if it >= 5:
            ts.append(e0.elapsed_time(e1) / 10)
    return statistics.median(ts) * 1e3


C = ext()
H, F = 4096, 11008
sync = torch.zeros(2, dtype=torch.int64, device="cuda")
for M in (1, 8):
    ctx = torch.randn(M, H, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(M, H, device="cuda", dtype=torch.bfloat16)
    wo = torch.randn(H, H, device="cuda", dtype=torch.bfloat16) * 0.02
    w1 = torch.randn(2 * F, H, device="cuda", dtype=torch.bfloat16) * 0.02
    w2 = torch.randn(H, F, device="cuda", dtype=torch.bfloat16) * 0.02
    g = torch.ones(H, device="cuda", dtype=torch.bfloat16)

    def three():
        h2 = C.skinny_norm_gemm(ctx, wo, None, 0.0, x)
        a = C.skinny_norm_glu(h2, w1, g, 1e-5, 0)
        return C.skinny_norm_gemm(a, w2, None, 0.0, h2)

    def fused(mode=0):
        return C.decode_mlp(ctx, x, wo, g, 1e-5, w1, w2, 0, sync, mode) if mode else \
            C.decode_mlp(ctx, x, wo, g, 1e-5, w1, w2, 0, sync)

    a3 = t(three)
    af = t(fused)
    gb = (H * H + 2 * F * H + H * F) * 2 / 1e9
    line = (f"M={M}: three launches {a3:.1f} us ({gb / a3 * 1e3:.2f} TB/s) | fused {af:.1f} us "
            f"({gb / af * 1e3:.2f} TB/s)")
    for mode in (1, 2, 3):
        try:
            am = t(lambda: fused(mode))
            line += f" | mode{mode} {am:.1f} us"
        except TypeError:
            break
    torch.cuda.synchronize()
    print(line + f" | timeouts {int(sync[1])}", flush=True)
