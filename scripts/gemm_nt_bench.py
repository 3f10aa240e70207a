"""A/B of the hand-written NT GEMM (csrc/gemm_nt.hip) against hipBLASLt
(torch.matmul) on the Llama-2-7B training shapes, interleaved in one process
(CDNA guide §5.4 rule 24), uniform-random operands (rule 25).

    python scripts/gemm_nt_bench.py [--m 16384] [--rounds 5] [--tp 1]
"""
import argparse
import json
import statistics

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=16384)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--ffn", type=int, default=11008)
    ap.add_argument("--qkv", type=int, default=12288)
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--json", default=None)
    ap.add_argument("--variants", default="4,8", help="NT GEMM kernel variants to time")
    args = ap.parse_args()
    from epfl_megatron_amd.ops._ext import ext
    C = ext()
    dev = "cuda"
    M, H, F, Q, tp = args.m, args.hidden, args.ffn // args.tp, args.qkv // args.tp, args.tp
    dt = torch.bfloat16

    def r(*s):
        return torch.empty(*s, device=dev, dtype=dt).uniform_(-1, 1)

    cases = []
    # (name, flops, torch_fn, hip_fn)
    def add_plain(name, n, k):
        a, b = r(M, k), r(n, k)
        out = torch.empty(M, n, device=dev, dtype=dt)
        cases.append((name, 2.0 * M * n * k,
                      lambda: torch.matmul(a, b.t(), out=out),
                      lambda: C.gemm_nt(a, b, out)))

    add_plain("fwd_qkv", Q, H)
    add_plain("fwd_o", H, H // tp)
    add_plain("fwd_fc2", H, F)
    add_plain("dgrad_qkv", H, Q)
    add_plain("dgrad_o", H // tp, H)
    add_plain("dgrad_fc1", H, 2 * F)
    # fc1 forward: hipBLASLt + glu_fwd vs fused
    x, w1 = r(M, H), r(2 * F, H)
    pre_o = torch.empty(M, 2 * F, device=dev, dtype=dt)
    cases.append(("fwd_fc1+glu", 2.0 * M * 2 * F * H,
                  lambda: C.glu_fwd(torch.matmul(x, w1.t(), out=pre_o), 0),
                  lambda: C.gemm_nt_glu(x, w1, 0)))
    # fc2 dgrad: hipBLASLt + glu_bwd vs fused
    dy, w2t, pre = r(M, H), r(F, H), r(M, 2 * F)
    da = torch.empty(M, F, device=dev, dtype=dt)
    cases.append(("dgrad_fc2+dglu", 2.0 * M * F * H,
                  lambda: C.glu_bwd(torch.matmul(dy, w2t.t(), out=da), pre, 0),
                  lambda: C.gemm_nt_dglu(dy, w2t, pre, 0)))
    # bare plain-GEMM reference for the glu shapes
    add_plain("fwd_fc1_plain", 2 * F, H)
    add_plain("dgrad_fc2_plain", F, H)

    variants = [int(v) for v in args.variants.split(",")]
    res = {c[0]: {"lt": [], **{v: [] for v in variants}} for c in cases}
    for _ in range(args.rounds):
        for name, fl, tf, hf in cases:
            res[name]["lt"].append(fl / timeit(tf, args.iters) / 1e9)
            for v in variants:
                C.gemm_nt_set_variant(v)
                res[name][v].append(fl / timeit(hf, args.iters) / 1e9)
    out = {}
    for name, fl, _, _ in cases:
        lt = statistics.median(res[name]["lt"])
        out[name] = {"hipblaslt_tflops": round(lt, 1)}
        line = f"{name:18s} hipBLASLt {lt:7.1f} TF/s"
        for v in variants:
            hp = statistics.median(res[name][v])
            out[name][f"hip{v}_tflops"] = round(hp, 1)
            line += f"   hip{v} {hp:7.1f} (x{hp / lt:.3f})"
        print(line, flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump({"M": M, "tp": tp, "cases": out}, f, indent=1)


if __name__ == "__main__":
    main()
