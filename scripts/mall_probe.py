"""Does a decode GEMM run faster when its weights were just read (MALL-warm)?
o_proj / QKV / fc1 skinny kernels at batch 1, timed (a) back to back (weights
warm in the 256 MB Infinity Cache), (b) after streaming 1 GiB of other data
(cold), (c) cold but with the weights read by torch.sum right before.
Usage: python scripts/mall_probe.py"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from epfl_megatron_amd.ops import decode_pack  # noqa: E402
from epfl_megatron_amd.ops._ext import ext  # noqa: E402


def main():
    C = ext()
    h, f = 4096, 11008
    dt = torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(0)
    wo = torch.randn(h, h, device="cuda", dtype=dt, generator=g) * 0.02
    wq = torch.randn(3 * h, h, device="cuda", dtype=dt, generator=g) * 0.02
    po, pq = decode_pack.packed(wo), decode_pack.packed(wq)
    x = torch.randn(1, h, device="cuda", dtype=dt, generator=g)
    res = torch.randn(1, h, device="cuda", dtype=dt, generator=g)
    lnw = torch.ones(h, device="cuda", dtype=dt)
    flush = torch.empty(1 << 29, device="cuda", dtype=torch.float16)  # 1 GiB
    cases = [("o_proj", po, lambda: C.skinny_norm_gemm(x, po, None, 0.0, res, True)),
             ("qkv", pq, lambda: C.skinny_norm_gemm(x, pq, lnw, 1e-5, None, True))]
    for name, w, fn in cases:
        out = {}
        for mode in ("warm", "cold", "cold+sum"):
            ts = []
            for it in range(25):
                if mode != "warm":
                    flush.add_(1)
                if mode == "cold+sum":
                    w.view(torch.int16).sum(dtype=torch.int32)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                if it >= 5:
                    ts.append(e0.elapsed_time(e1) * 1e3)
            out[mode] = statistics.median(ts)
        print(f"{name}: " + ", ".join(f"{k} {v:.1f} us" for k, v in out.items()), flush=True)


if __name__ == "__main__":
    main()
