"""FlashAttention forward diagnosis: where does the short-sequence rate go?

Times the forward kernel alone (20 back-to-back launches per sample, median of
5) at a constant 16k tokens for s = 1k / 2k / 4k / 8k, causal and non-causal,
on uniform random data.  If the non-causal rate is flat in s while the causal
one falls at small s, the loss is in the causal edge (diagonal tiles, load
balance), not in the per-tile pipeline.

    python scripts/fa_diag.py [--json out.json]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--heads", type=int, default=32)
    ap.add_argument("--hd", type=int, default=128)
    args = ap.parse_args()
    from epfl_megatron_amd.ops._ext import ext
    C = ext()
    nq, hd = args.heads, args.hd
    res = []
    for s in (1024, 2048, 4096, 8192):
        b = max(1, args.tokens // s)
        q = torch.empty(b, s, nq, hd, device="cuda", dtype=torch.bfloat16).uniform_(-2, 2)
        k = torch.empty_like(q).uniform_(-2, 2)
        v = torch.empty_like(q).uniform_(-1, 1)
        out = torch.empty_like(q)
        lse = torch.empty(b, nq, s, device="cuda", dtype=torch.float32)
        qs = [q.stride(0), q.stride(1), q.stride(2), q.stride(2)]
        ks = [k.stride(0), k.stride(1), k.stride(2)]
        os_ = [out.stride(0), out.stride(1), out.stride(2)]
        for causal in (True, False):
            def run():
                C.flash_attn_fwd(q, k, v, out, lse, b, s, s, nq, nq, hd, qs, ks, ks, os_, causal,
                                 hd ** -0.5, None, None, None, None)
            run()
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    run()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) / 20)
            ms = statistics.median(ts)
            fl = 4.0 * b * nq * s * s * hd * (0.5 if causal else 1.0)
            tf = fl / ms / 1e9
            r = {"b": b, "s": s, "causal": causal, "us": round(ms * 1e3, 1), "tflops": round(tf, 1)}
            res.append(r)
            print(f"b={b:3d} s={s:5d} causal={int(causal)}  {ms * 1e3:8.1f} us  {tf:6.1f} TF/s",
                  flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
