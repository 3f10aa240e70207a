"""Decode-batch GEMM timing: csrc/skinny_gemm.hip vs torch.matmul (hipBLASLt) on the
Llama-2-7B projection shapes.  Usage: python scripts/skinny_bench.py"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from epfl_megatron_amd.ops._ext import ext  # noqa: E402


def t(fn):
    ts = []
    for it in range(25):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        if it >= 5:
            ts.append(e0.elapsed_time(e1))
    return statistics.median(ts) * 1e3


for M in (1, 8, 16):
    for N, K in ((12288, 4096), (4096, 4096), (22016, 4096), (4096, 11008), (32000, 4096)):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        a = t(lambda: ext().skinny_gemm(x, w))
        b = t(lambda: torch.matmul(x, w.t()))
        gb = N * K * 2 / 1e9
        print(f"M={M} N={N} K={K}: skinny {a:.1f} us ({gb / a * 1e3:.2f} TB/s) | hipBLASLt {b:.1f} us "
              f"({gb / b * 1e3:.2f} TB/s) -> {b / a:.2f}x", flush=True)
