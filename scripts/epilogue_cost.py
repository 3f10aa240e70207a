"""What the GEMM epilogues cost in the training step's cache state.

Isolated benchmarks re-run one GEMM on the same output buffer, so its fp32
main_grad block (wgrad) or its saved pre-activation (dGLU) sits in the 256 MiB
Infinity Cache; in the step every layer's buffers are cold.  This times each
7B shape per call, hot (back to back) and cold (a 1 GiB write between calls
evicts the Infinity Cache), for:

  wgrad   accumulate (fp32 read-modify-write of G) vs store-only (first
          micro-batch), so acc - store = the read half of the epilogue;
  NT      plain product vs fused SwiGLU (fc1 forward) and fused dSwiGLU
          (fc2 dgrad: reads the saved pre-activation, writes d(pre)).

    python scripts/epilogue_cost.py [--iters 6]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def per_call(fn, iters, flush=None):
    ts = []
    for _ in range(iters + 1):
        if flush is not None:
            flush()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    return statistics.median(ts[1:])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--m", type=int, default=16384)
    args = ap.parse_args()
    from epfl_megatron_amd.ops._ext import ext
    C = ext()
    M, dt = args.m, torch.bfloat16
    junk = torch.empty(1 << 28, device="cuda", dtype=torch.float32)

    def flush():
        junk.fill_(1.0)

    def r(*s):
        return torch.empty(*s, device="cuda", dtype=dt).uniform_(-1, 1)

    print("wgrad (us/call, TF/s)            hot-acc    cold-acc   cold-store  hot-store", flush=True)
    for name, (N, K) in {"qkv": (12288, 4096), "dense": (4096, 4096), "fc1": (22016, 4096),
                         "fc2": (4096, 11008)}.items():
        dY, X = r(M, N), r(M, K)
        G = torch.zeros(N, K, device="cuda", dtype=torch.float32)
        fl = 2.0 * M * N * K
        row = []
        for acc, fl_ in ((True, None), (True, flush), (False, flush), (False, None)):
            us = per_call(lambda: C.wgrad_gemm(dY, X, G, acc), args.iters, fl_)
            row.append(f"{us:8.0f} {fl / us / 1e6:6.0f}")
        print(f"  {name:6s} M{M} N{N} K{K}  " + "  ".join(row), flush=True)
        del dY, X, G

    print("NT (us/call, TF/s)                   hot        cold", flush=True)
    H, F = 4096, 11008
    x, w1 = r(M, H), r(2 * F, H)
    out1 = torch.empty(M, 2 * F, device="cuda", dtype=dt)
    dy, w2t, pre = r(M, H), r(F, H), r(M, 2 * F)
    out2 = torch.empty(M, F, device="cuda", dtype=dt)
    cases = [
        ("fc1 plain", 2.0 * M * 2 * F * H, lambda: C.gemm_nt(x, w1, out1)),
        ("fc1 +GLU", 2.0 * M * 2 * F * H, lambda: C.gemm_nt_glu(x, w1, 0)),
        ("fc2dg plain", 2.0 * M * F * H, lambda: C.gemm_nt(dy, w2t, out2)),
        ("fc2dg +dGLU", 2.0 * M * F * H, lambda: C.gemm_nt_dglu(dy, w2t, pre, 0)),
        ("fc1 hipBLASLt", 2.0 * M * 2 * F * H, lambda: torch.matmul(x, w1.t(), out=out1)),
    ]
    for name, fl, fn in cases:
        hot = per_call(fn, args.iters)
        cold = per_call(fn, args.iters, flush)
        print(f"  {name:14s} {hot:8.0f} {fl / hot / 1e6:6.0f}   {cold:8.0f} {fl / cold / 1e6:6.0f}",
              flush=True)


if __name__ == "__main__":
    main()
