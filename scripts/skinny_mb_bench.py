"""Decode-batch fused skinny GEMMs at 16 / 24 / 32 rows (one vs two 16-row
blocks per W fragment) vs hipBLASLt, Llama-2-7B decode shapes, decode-packed
weights.  Usage: python scripts/skinny_mb_bench.py [--rows 16,24,32]"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from epfl_megatron_amd.ops import decode_pack  # noqa: E402
from epfl_megatron_amd.ops._ext import ext  # noqa: E402


def t(fn):
    ts = []
    for it in range(30):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        if it >= 5:
            ts.append(e0.elapsed_time(e1))
    return statistics.median(ts) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="16,24,32")
    a = ap.parse_args()
    C = ext()
    h, f = 4096, 11008
    dt = torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(0)
    wqkv = torch.randn(3 * h, h, device="cuda", dtype=dt, generator=g) * 0.02
    wo = torch.randn(h, h, device="cuda", dtype=dt, generator=g) * 0.02
    w1 = torch.randn(2 * f, h, device="cuda", dtype=dt, generator=g) * 0.02
    w2 = torch.randn(h, f, device="cuda", dtype=dt, generator=g) * 0.02
    lnw = torch.ones(h, device="cuda", dtype=dt)
    tail = C.skinny_glu_half_tail(f, h, True)
    pq, po, p2 = decode_pack.packed(wqkv), decode_pack.packed(wo), decode_pack.packed(w2)
    p1 = decode_pack.packed(w1, glu=True, half_tail=tail)
    for m in [int(x) for x in a.rows.split(",")]:
        x = torch.randn(m, h, device="cuda", dtype=dt, generator=g)
        xf = torch.randn(m, f, device="cuda", dtype=dt, generator=g)
        res = torch.randn(m, h, device="cuda", dtype=dt, generator=g)
        cases = [
            ("qkv norm", wqkv, lambda: C.skinny_norm_gemm(x, pq, lnw, 1e-5, None, True),
             lambda: torch.matmul(x, wqkv.t())),
            ("o_proj +res", wo, lambda: C.skinny_norm_gemm(x, po, None, 0.0, res, True),
             lambda: torch.matmul(x, wo.t())),
            ("fc1 norm+swiglu", w1, lambda: C.skinny_norm_glu(x, p1, lnw, 1e-5, 0, True, tail),
             lambda: torch.matmul(x, w1.t())),
            ("fc2 +res (K=11008)", w2, lambda: C.skinny_norm_gemm(xf, p2, None, 0.0, res, True),
             lambda: torch.matmul(xf, w2.t())),
        ]
        for name, w, sk, bl in cases:
            a_us, b_us = t(sk), t(bl)
            gb = w.numel() * 2 / 1e9
            print(f"M={m:2d} {name:20s}: skinny {a_us:6.1f} us ({gb / a_us * 1e3:.2f} TB/s) | "
                  f"hipBLASLt {b_us:6.1f} us ({gb / b_us * 1e3:.2f} TB/s) -> {b_us / a_us:.2f}x",
                  flush=True)


if __name__ == "__main__":
    main()
