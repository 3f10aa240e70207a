"""Decode attention timing: split-key decode kernel vs the FlashAttention
forward kernel on one query token (1 GPU).  Usage: python scripts/decode_bench.py"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from epfl_megatron_amd.ops import attention as A  # noqa: E402


def bench(b, sk, nq, nkv, hd):
    torch.manual_seed(0)
    kmem = torch.randn(sk, b, nkv, hd, device="cuda", dtype=torch.bfloat16)
    vmem = torch.randn(sk, b, nkv, hd, device="cuda", dtype=torch.bfloat16)
    q = torch.randn(b, 1, nq, hd, device="cuda", dtype=torch.bfloat16)
    keys, vals = kmem.transpose(0, 1), vmem.transpose(0, 1)
    scale = hd ** -0.5
    out = {}
    for name, fn in (("decode", lambda: A._flash_decode(q, keys, vals, scale)),
                     ("fa_fwd", lambda: A._FlashFn.apply(q, keys, vals, True, scale))):
        ts = []
        with torch.no_grad():
            for it in range(23):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                if it >= 3:
                    ts.append(e0.elapsed_time(e1))
        out[name] = statistics.median(ts) * 1e3
    kv_bytes = 2 * b * sk * nkv * hd * 2
    print(f"b={b} sk={sk} nq={nq} nkv={nkv} hd={hd}: decode {out['decode']:.1f} us "
          f"({kv_bytes / out['decode'] / 1e3:.0f} GB/s of KV) | fa_fwd {out['fa_fwd']:.1f} us "
          f"-> {out['fa_fwd'] / out['decode']:.1f}x", flush=True)


if __name__ == "__main__":
    for sh in ((1, 2048, 32, 32, 128), (8, 2048, 32, 32, 128), (1, 4096, 64, 8, 128),
               (16, 4096, 64, 8, 128), (4, 2048, 71, 1, 64), (1, 256, 32, 32, 128),
               (8, 256, 32, 32, 128), (32, 256, 32, 32, 128)):
        bench(*sh)
