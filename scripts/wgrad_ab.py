"""Interleaved A/B (one process, CDNA guide rule 24) of the two wgrad kernels
(csrc/gemm_wgrad.hip: 8 = 8-wave ping-pong wgrad_k, 4 = persistent 4-wave
wgrad4_k) and hipBLASLt on the Llama-2-7B micro-batch shapes (M = 16384
tokens), fp32 accumulate into G; both kernels are first checked against an
fp32 oracle."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from epfl_megatron_amd.ops._ext import ext  # noqa: E402

SHAPES = {"qkv": (12288, 4096), "dense": (4096, 4096), "fc1": (22016, 4096),
          "fc2": (4096, 11008), "lm_head": (32000, 4096)}


def _t(fn, iters=8):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    C = ext()
    torch.manual_seed(0)
    for v in (4, 8):
        C.wgrad_set_variant(v)
        for (M, N, K) in [(4096, 768, 512), (8192, 512, 1280), (2048, 2752, 4096)]:
            dY = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
            X = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            G = torch.randn(N, K, device="cuda", dtype=torch.float32)
            ref = G + dY.float().t() @ X.float()
            C.wgrad_gemm(dY, X, G, True)
            err = ((G - ref).abs().max() / ref.abs().max()).item()
            assert err < 1e-4, (v, M, N, K, err)
    print("numerics ok (variants 4 and 8)", flush=True)
    M = 16384
    for name, (N, K) in SHAPES.items():
        dY = torch.empty(M, N, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        X = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        G = torch.zeros(N, K, device="cuda", dtype=torch.float32)
        fl = 2.0 * M * N * K
        r = {"v8": [], "v4": [], "hipblaslt": []}
        for _ in range(5):
            for v in (8, 4):
                C.wgrad_set_variant(v)
                r[f"v{v}"].append(fl / _t(lambda: C.wgrad_gemm(dY, X, G, True)) / 1e12)
            r["hipblaslt"].append(fl / _t(lambda: C.lt_gemm(dY, True, X, False, G, 1.0, 1.0, -1)) / 1e12)
        med = {k: statistics.median(v) for k, v in r.items()}
        print(f"{name:8s} " + "  ".join(f"{k} {v:7.1f}" for k, v in med.items()) +
              f" TF/s  (v4/v8 x{med['v4'] / med['v8']:.3f})", flush=True)
    C.wgrad_set_variant(4)  # the default


if __name__ == "__main__":
    main()
